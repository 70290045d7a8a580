// Launch-bound co-tenancy on one MI355X: N tenants each launching a stream of tiny kernels,
// either as N processes (N HSA processes: N VMIDs on the GPU's hardware scheduler) or as N
// threads of one process, each with a stream of its own (one process, N queues). Separates a
// cross-process effect (how the scheduler serves several processes' queues) from a
// cross-queue one (profiles/r5k: four LSTM pods run their ~5 us kernels 13-22x longer than
// two).
//
//   cotenancy_probe procs|streams N SECONDS [SPIN_US] [GRID] [WAIT] [PIN]  -> one JSON line
//
// WAIT: how a tenant waits for its stream - spin (hipStreamSynchronize with HIP's default
// scheduling: the runtime spins), block (hipDeviceScheduleBlockingSync: the runtime sleeps in
// the driver until an interrupt), poll (hipStreamQuery every 20 us with a nanosleep between:
// no runtime wait at all). PIN: none, same (tenant i on the i-th physical core of NUMA node
// 0), split (tenant i on node i mod 2), gpu (all on the GPU's own node). Per tenant the probe
// also reports the host time inside the launch call and inside one wait, so the host call
// that grows with co-tenancy is named without a tracer in the way.
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
  double launch_us = 0, wait_us = 0;  // mean host time inside one launch call / one wait
  long kernels = 0;
  int cpu = -1, node = -1;
  bool ok = false;
};

enum class Wait { kSpin, kBlock, kPoll };

double mono_us() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return ts.tv_sec * 1e6 + ts.tv_nsec * 1e-3;
}

std::vector<int> parse_cpulist(const std::string& txt) {
  std::vector<int> out;
  size_t i = 0;
  while (i < txt.size()) {
    char* end = nullptr;
    long lo = strtol(txt.c_str() + i, &end, 10);
    if (end == txt.c_str() + i) break;
    long hi = lo;
    i = end - txt.c_str();
    if (i < txt.size() && txt[i] == '-') {
      hi = strtol(txt.c_str() + i + 1, &end, 10);
      i = end - txt.c_str();
    }
    for (long c = lo; c <= hi; c++) out.push_back((int)c);
    while (i < txt.size() && (txt[i] == ',' || txt[i] == '\n')) i++;
  }
  return out;
}

std::string read_text(const std::string& path) {
  FILE* f = fopen(path.c_str(), "r");
  if (!f) return "";
  char buf[4096] = {0};
  const size_t got = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  return std::string(buf, got);
}

// The allowed physical cores (first SMT sibling) of NUMA node `node`.
std::vector<int> node_cores(int node) {
  cpu_set_t allowed;
  CPU_ZERO(&allowed);
  sched_getaffinity(0, sizeof(allowed), &allowed);
  std::vector<int> out;
  for (int c : parse_cpulist(read_text("/sys/devices/system/node/node" + std::to_string(node) + "/cpulist"))) {
    if (c < 0 || c >= CPU_SETSIZE || !CPU_ISSET(c, &allowed)) continue;
    const std::vector<int> sib =
        parse_cpulist(read_text("/sys/devices/system/cpu/cpu" + std::to_string(c) + "/topology/thread_siblings_list"));
    if (sib.empty() || sib[0] == c) out.push_back(c);
  }
  return out;
}

int gpu_node() {
  // The first KFD GPU node's NUMA node (its PCI device's numa_node), 0 if unknown.
  for (int i = 0; i < 64; i++) {
    const std::string t = read_text("/sys/class/kfd/kfd/topology/nodes/" + std::to_string(i) + "/properties");
    if (t.empty() || t.find("simd_count 0\n") != std::string::npos) continue;  // none, or a CPU node
    const size_t l = t.find("location_id "), d = t.find("domain ");
    if (l == std::string::npos) continue;
    const unsigned loc = (unsigned)strtoul(t.c_str() + l + 12, nullptr, 10);
    const unsigned dom = d == std::string::npos ? 0 : (unsigned)strtoul(t.c_str() + d + 7, nullptr, 10);
    char bdf[32];
    snprintf(bdf, sizeof(bdf), "%04x:%02x:%02x.%x", dom, (loc >> 8) & 0xff, (loc >> 3) & 0x1f, loc & 7);
    const std::string n = read_text(std::string("/sys/bus/pci/devices/") + bdf + "/numa_node");
    return n.empty() ? 0 : std::max(0, atoi(n.c_str()));
  }
  return 0;
}

// The CPU tenant i runs on under `pin` (-1: unpinned).
int pin_cpu(const std::string& pin, int i) {
  if (pin == "none" || pin.empty()) return -1;
  const int node = pin == "split" ? i % 2 : pin == "gpu" ? gpu_node() : 0;
  const int k = pin == "split" ? i / 2 : i;
  const std::vector<int> cores = node_cores(node);
  return cores.empty() ? -1 : cores[k % cores.size()];
}

void pin_to(int cpu) {
  if (cpu < 0) return;
  cpu_set_t set;
  CPU_ZERO(&set);
  CPU_SET(cpu, &set);
  sched_setaffinity(0, sizeof(set), &set);  // the calling thread
}

int node_of(int cpu) {
  for (int n = 0; n < 16; n++) {
    const std::vector<int> cs = parse_cpulist(read_text("/sys/devices/system/node/node" + std::to_string(n) + "/cpulist"));
    if (std::find(cs.begin(), cs.end(), cpu) != cs.end()) return n;
  }
  return -1;
}

hipError_t wait_stream(hipStream_t s, Wait w) {
  if (w != Wait::kPoll) return hipStreamSynchronize(s);
  for (;;) {
    const hipError_t e = hipStreamQuery(s);
    if (e != hipErrorNotReady) return e;
    struct timespec ts = {0, 20000};
    nanosleep(&ts, nullptr);
  }
}

// One tenant: its own stream, launches for `seconds` starting at `start` (CLOCK_REALTIME).
Result tenant(double start, double seconds, double spin_us, int grid, Wait w, int cpu) {
  Result r;
  pin_to(cpu);
  if (w == Wait::kBlock) (void)hipSetDeviceFlags(hipDeviceScheduleBlockingSync);
  int rate_khz = 0;
  if (hipDeviceGetAttribute(&rate_khz, hipDeviceAttributeWallClockRate, 0) != hipSuccess || rate_khz <= 0) return r;
  const uint64_t ticks = (uint64_t)(spin_us * rate_khz / 1000.0);
  hipStream_t s;
  uint64_t* out = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return r;
  if (hipMalloc(&out, sizeof(uint64_t) * 2 * kRing) != hipSuccess) return r;
  for (int i = 0; i < 64; i++) spin_kernel<<<grid, 64, 0, s>>>(ticks, out, i % kRing);  // warm-up
  if (wait_stream(s, w) != hipSuccess) return r;
  while (realtime_s() < start) usleep(200);
  const double t0 = realtime_s();
  long n = 0, waits = 0;
  double in_launch = 0, in_wait = 0;
  while (realtime_s() - t0 < seconds) {
    const double a = mono_us();
    spin_kernel<<<grid, 64, 0, s>>>(ticks, out, (int)(n % kRing));
    const double b = mono_us();
    in_launch += b - a;
    if (++n % 8 == 0) {
      (void)wait_stream(s, w);
      in_wait += mono_us() - b;
      waits++;
    }
  }
  (void)wait_stream(s, w);
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
  r.launch_us = n ? in_launch / n : 0;
  r.wait_us = waits ? in_wait / waits : 0;
  r.cpu = sched_getcpu();
  r.node = node_of(r.cpu);
  r.ok = true;
  (void)hipFree(out);
  (void)hipStreamDestroy(s);
  return r;
}

// A tenant that sets up exactly like an active one (HIP, its stream's hardware queue, the
// warm-up kernels) and then sleeps through the window: does a process whose queues are mapped
// but idle slow the active ones?
void idle_tenant(double start, double seconds, int grid, int cpu) {
  pin_to(cpu);
  hipStream_t s;
  uint64_t* out = nullptr;
  if (hipStreamCreateWithFlags(&s, hipStreamNonBlocking) != hipSuccess) return;
  if (hipMalloc(&out, sizeof(uint64_t) * 2 * kRing) != hipSuccess) return;
  for (int i = 0; i < 64; i++) spin_kernel<<<grid, 64, 0, s>>>(1000, out, i % kRing);
  (void)hipStreamSynchronize(s);
  while (realtime_s() < start + seconds + 0.5) usleep(10000);
  (void)hipFree(out);
  (void)hipStreamDestroy(s);
}

void print_result(FILE* f, const Result& r) {
  fprintf(f, "{\"ok\": %s, \"kernels\": %ld, \"kps\": %.1f, \"p50_us\": %.2f, \"p90_us\": %.2f, \"max_us\": %.2f, "
             "\"launch_us\": %.3f, \"wait_us\": %.2f, \"cpu\": %d, \"node\": %d}",
          r.ok ? "true" : "false", r.kernels, r.kps, r.p50_us, r.p90_us, r.max_us, r.launch_us, r.wait_us, r.cpu, r.node);
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
    fprintf(stderr, "usage: %s procs|streams N SECONDS [SPIN_US] [GRID] [spin|block|poll] [none|same|split|gpu] [IDLE]\n",
            argv[0]);
    return 2;
  }
  const std::string mode = argv[1];
  const int n = std::max(1, std::min(64, atoi(argv[2])));
  const double seconds = atof(argv[3]);
  const double spin_us = argc > 4 ? atof(argv[4]) : 5.0;
  const int grid = argc > 5 ? std::max(1, atoi(argv[5])) : 4;
  const std::string wait_s = argc > 6 ? argv[6] : "spin";
  const std::string pin = argc > 7 ? argv[7] : "none";
  const Wait w = wait_s == "block" ? Wait::kBlock : wait_s == "poll" ? Wait::kPoll : Wait::kSpin;
  if (wait_s != "spin" && wait_s != "block" && wait_s != "poll") {
    fprintf(stderr, "unknown wait %s\n", wait_s.c_str());
    return 2;
  }
  const int idle = argc > 8 ? std::max(0, std::min(32, atoi(argv[8]))) : 0;  // procs mode: idle co-tenants
  std::vector<int> cpus(n + idle);
  for (int i = 0; i < n + idle; i++) cpus[i] = pin_cpu(pin, i);
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
        Result r = tenant(start, seconds, spin_us, grid, w, cpus[i]);
        if (write(p[1], &r, sizeof(r)) != (ssize_t)sizeof(r)) _exit(3);
        _exit(r.ok ? 0 : 1);
      }
      close(p[1]);
      fds[i] = p[0];
      kids[i] = c;
    }
    std::vector<pid_t> idlers;
    for (int i = 0; i < idle; i++) {
      pid_t c = fork();
      if (c == 0) {
        idle_tenant(start, seconds, grid, cpus[n + i]);
        _exit(0);
      }
      if (c > 0) idlers.push_back(c);
    }
    for (int i = 0; i < n; i++) {
      if (read(fds[i], &res[i], sizeof(Result)) != (ssize_t)sizeof(Result)) res[i] = Result();
      close(fds[i]);
      int st = 0;
      waitpid(kids[i], &st, 0);
    }
    for (pid_t c : idlers) {
      int st = 0;
      waitpid(c, &st, 0);
    }
  } else if (mode == "streams") {
    std::vector<std::thread> th;
    for (int i = 0; i < n; i++) th.emplace_back([&, i] { res[i] = tenant(start, seconds, spin_us, grid, w, cpus[i]); });
    for (auto& t : th) t.join();
  } else {
    fprintf(stderr, "unknown mode %s\n", mode.c_str());
    return 2;
  }
  double agg = 0;
  for (const Result& r : res) agg += r.kps;
  printf("{\"mode\": \"%s\", \"tenants\": %d, \"idle\": %d, \"wait\": \"%s\", \"pin\": \"%s\", \"seconds\": %.1f, \"spin_us\": %.1f, "
         "\"grid\": %d, \"aggregate_kps\": %.1f, "
         "\"amdgpu\": {\"hws_max_conc_proc\": %s, \"sched_policy\": %s, \"cwsr_enable\": %s, \"mes\": %s, "
         "\"sched_hw_submission\": %s}, \"per_tenant\": [",
         mode.c_str(), n, mode == "procs" ? idle : 0, wait_s.c_str(), pin.c_str(), seconds, spin_us, grid, agg, module_param("hws_max_conc_proc").c_str(),
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
