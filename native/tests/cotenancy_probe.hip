// Launch-bound co-tenancy on one MI355X: N tenants each launching a stream of tiny kernels,
// either as N processes (N HSA processes: N VMIDs on the GPU's hardware scheduler) or as N
// threads of one process, each with a stream of its own (one process, N queues). Separates a
// cross-process effect (how the scheduler serves several processes' queues) from a
// cross-queue one (profiles/r5k: four LSTM pods run their ~5 us kernels 13-22x longer than
// two).
//
//   cotenancy_probe procs|streams N SECONDS [SPIN_US] [GRID]  -> one JSON line
//
// Each kernel spins on the GPU's constant-rate wall clock for SPIN_US and records its own
// start and end, so a kernel that is descheduled mid-flight (its waves saved and restored by
// the scheduler, or starved of a dispatch slot) shows up as a duration longer than SPIN_US,
// whatever the launch rate. Each tenant synchronises every 8 launches (as a launch-bound
// framework does). Reported per tenant: kernels/s, and the median / p90 / max kernel duration
// over its last 2048 kernels; plus the amdgpu module parameters that shape the scheduling
// (read from /sys/module/amdgpu/parameters when readable).
//
// Processes are forked before any HIP call (HIP is not fork-safe); all tenants start at the
// same CLOCK_REALTIME instant. Every kernel's spin loop is bounded (an iteration cap), so the
// grid drains even if the clock misbehaves.
#include <hip/hip_runtime.h>
#include <sched.h>
#include <sys/wait.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

namespace {

constexpr int kRing = 2048;  // kernels whose durations are kept, per tenant

__global__ void spin_kernel(uint64_t ticks, uint64_t* out, int slot) {
  const uint64_t t0 = wall_clock64();
  uint64_t t = t0;
  for (int it = 0; t - t0 < ticks && it < (1 << 22); it++) t = wall_clock64();
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    out[2 * slot] = t0;
    out[2 * slot + 1] = t;
  }
}

double realtime_s() {
  struct timespec ts;
  clock_gettime(CLOCK_REALTIME, &ts);
  return ts.tv_sec + ts.tv_nsec * 1e-9;
}

struct Result {
  double kps = 0, p50_us = 0, p90_us = 0, max_us = 0;
  long kernels = 0;
  int cpu = -1;
  bool ok = false;
};

// One tenant: its own stream, launches for `seconds` starting at `start` (CLOCK_REALTIME).
Result tenant(double start, double seconds, double spin_us, int grid) {
  Result r;
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || rate_khz <= 0) return r;
  const uint64_t ticks = (uint64_t)(spin_us * rate_khz / 1000.0);
  hipStream_t s;
  uint64_t* out = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return r;
  if (hipMalloc(&out, sizeof(uint64_t) * 2 * kRing) != hipSuccess) return r;
  for (int i = 0; i < 64; i++) spin_kernel<<<grid, 64, 0, s>>>(ticks, out, i % kRing);  // warm-up
  if (hipStreamSynchronize(s) != hipSuccess) return r;
  while (realtime_s() < start) usleep(200);
  const double t0 = realtime_s();
  long n = 0;
  while (realtime_s() - t0 < seconds) {
    spin_kernel<<<grid, 64, 0, s>>>(ticks, out, (int)(n % kRing));
    if (++n % 8 == 0) (void)hipStreamSynchronize(s);
  }
  (void)hipStreamSynchronize(s);
  const double dt = realtime_s() - t0;
  std::vector<uint64_t> h(2 * kRing);
  if (hipMemcpy(h.data(), out, sizeof(uint64_t) * h.size(), hipMemcpyDeviceToHost) != hipSuccess) return r;
  std::vector<double> d;
  for (long i = 0; i < std::min<long>(n, kRing); i++)
    if (h[2 * i + 1] >= h[2 * i]) d.push_back((h[2 * i + 1] - h[2 * i]) * 1000.0 / rate_khz);
  std::sort(d.begin(), d.end());
  if (!d.empty()) {
    r.p50_us = d[d.size() / 2];
    r.p90_us = d[d.size() * 9 / 10];
    r.max_us = d.back();
  }
  r.kernels = n;
  r.kps = n / dt;
  r.cpu = sched_getcpu();
  r.ok = true;
  (void)hipFree(out);
  (void)hipStreamDestroy(s);
  return r;
}

void print_result(FILE* f, const Result& r) {
  fprintf(f, "{\"ok\": %s, \"kernels\": %ld, \"kps\": %.1f, \"p50_us\": %.2f, \"p90_us\": %.2f, \"max_us\": %.2f, "
             "\"cpu\": %d}",
          r.ok ? "true" : "false", r.kernels, r.kps, r.p50_us, r.p90_us, r.max_us, r.cpu);
}

std::string module_param(const char* name) {
  std::string p = std::string("/sys/module/amdgpu/parameters/") + name;
  FILE* f = fopen(p.c_str(), "r");
  if (!f) return "null";
  char buf[64] = {0};
  const size_t got = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[got] = 0;
  for (char* c = buf; *c; c++)
    if (*c == '\n' || *c == '"') *c = 0;
  return std::string("\"") + buf + "\"";
}

}  // namespace

int main(int argc, char** argv) {
  if (argc < 4) {
    fprintf(stderr, "usage: %s procs|streams N SECONDS [SPIN_US] [GRID]\n", argv[0]);
    return 2;
  }
  const std::string mode = argv[1];
  const int n = std::max(1, std::min(64, atoi(argv[2])));
  const double seconds = atof(argv[3]);
  const double spin_us = argc > 4 ? atof(argv[4]) : 5.0;
  const int grid = argc > 5 ? std::max(1, atoi(argv[5])) : 4;
  const double start = realtime_s() + 3.0 + 0.1 * n;  // every tenant warmed up by then
  std::vector<Result> res(n);
  if (mode == "procs") {
    std::vector<int> fds(n);
    std::vector<pid_t> kids(n);
    for (int i = 0; i < n; i++) {
      int p[2];
      if (pipe(p) != 0) return 1;
      pid_t c = fork();
      if (c == 0) {
        close(p[0]);
        Result r = tenant(start, seconds, spin_us, grid);
        if (write(p[1], &r, sizeof(r)) != (ssize_t)sizeof(r)) _exit(3);
        _exit(r.ok ? 0 : 1);
      }
      close(p[1]);
      fds[i] = p[0];
      kids[i] = c;
    }
    for (int i = 0; i < n; i++) {
      if (read(fds[i], &res[i], sizeof(Result)) != (ssize_t)sizeof(Result)) res[i] = Result();
      close(fds[i]);
      int st = 0;
      waitpid(kids[i], &st, 0);
    }
  } else if (mode == "streams") {
    std::vector<std::thread> th;
    for (int i = 0; i < n; i++) th.emplace_back([&, i] { res[i] = tenant(start, seconds, spin_us, grid); });
    for (auto& t : th) t.join();
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  double agg = 0;
  for (const Result& r : res) agg += r.kps;
  printf("{\"mode\": \"%s\", \"tenants\": %d, \"seconds\": %.1f, \"spin_us\": %.1f, \"grid\": %d, \"aggregate_kps\": %.1f, "
         "\"amdgpu\": {\"hws_max_conc_proc\": %s, \"sched_policy\": %s, \"cwsr_enable\": %s, \"mes\": %s, "
         "\"sched_hw_submission\": %s}, \"per_tenant\": [",
         mode.c_str(), n, seconds, spin_us, grid, agg, module_param("hws_max_conc_proc").c_str(),
         module_param("sched_policy").c_str(), module_param("cwsr_enable").c_str(), module_param("mes").c_str(),
         module_param("sched_hw_submission").c_str());
  for (int i = 0; i < n; i++) {
    if (i) printf(", ");
    print_result(stdout, res[i]);
  }
  printf("]}\n");
  for (const Result& r : res)
    if (!r.ok) return 1;
  return 0;
}
