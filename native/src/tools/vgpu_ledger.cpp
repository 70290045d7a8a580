// vgpu-ledger: the node's GPU-time ledger daemon (see vgpu/ledger.h).
//
// Started by the device plugin with --ledger (plugin/main.py) next to the board directory.
// Every period it reads KFD cu_occupancy once for each process on each GPU that a live
// vGPU container has on the board, and integrates each process's processor-sharing
// charge from that one snapshot into <board>/ledger.<gpu_id> (root-owned, 0644: the
// containers mount the directory read-only). GPUs without limited containers cost
// nothing.
//
// One sampling thread per GPU: an occupancy read costs the GPU it walks, not the node, so
// each GPU's period is its own - it stretches only when that GPU's reads per base period
// exceed the read budget (ratelimit.h sample_period_ns), never because other GPUs of the
// node are busy too. An 8-GPU node at split 16 (128 processes) keeps the 1 ms period on every
// GPU (tests/test_multigpu.py); a single loop over every GPU would stretch it to 4 ms.
//
//   vgpu-ledger --dir <board dir> [--period-us 1000] [--read-budget 32] [--samples N] [--gpu ID]...
//
// --gpu samples that KFD gpu_id whether or not a container lists it (tests, operators).
// VGPU_KFD_ROOT points it at a fake KFD tree (tests). It exits with its parent.
#include <fcntl.h>
#include <signal.h>
#include <sys/mman.h>
#include <sys/prctl.h>
#include <sys/stat.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <set>
#include <string>
#include <thread>
#include <vector>

#include "vgpu/board.h"
#include "vgpu/kfd.h"
#include "vgpu/ledger.h"
#include "vgpu/ratelimit.h"

using namespace vgpu;

namespace {

volatile sig_atomic_t g_stop = 0;
void on_signal(int) { g_stop = 1; }

// Entries of a PID that left the GPU are kept this long (a container's last charge is
// read after its process exits), then reused.
constexpr uint64_t kForgetNs = 2'000'000'000ull;

struct Gpu {
  uint32_t gpu_id = 0;
  LedgerFile* f = nullptr;
  std::vector<int> pids;               // sampling thread's copy
  std::map<int, int64_t> prev_ppm;    // share at the previous sample, parts per million
  std::map<int, uint64_t> gone_since;  // entry PIDs no longer on the GPU
  uint64_t last_ns = 0;
  // Shared with the board thread: the GPU's current processes, and the stop request.
  std::mutex mu;
  std::vector<int> next_pids;
  std::atomic<bool> stop{false};
  std::thread th;
};

LedgerFile* create_ledger(const std::string& dir, uint32_t gpu_id) {
  const std::string path = ledger_path(dir, gpu_id);
  const std::string tmp = path + ".tmp";
  int fd = ::open(tmp.c_str(), O_RDWR | O_CREAT | O_TRUNC | O_CLOEXEC, 0644);
  if (fd < 0) return nullptr;
  fchmod(fd, 0644);  // readable by every container whatever the daemon's umask
  if (ftruncate(fd, sizeof(LedgerFile)) != 0) {
    ::close(fd);
    return nullptr;
  }
  void* p = mmap(nullptr, sizeof(LedgerFile), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
  ::close(fd);
  if (p == MAP_FAILED) return nullptr;
  LedgerFile* f = static_cast<LedgerFile*>(p);
  f->gpu_id = gpu_id;
  f->version = kLedgerVersion;
  std::atomic_thread_fence(std::memory_order_release);
  f->magic = kLedgerMagic;
  // Readers map the final name only once it is complete.
  if (rename(tmp.c_str(), path.c_str()) != 0) {
    munmap(p, sizeof(LedgerFile));
    return nullptr;
  }
  return f;
}

LedgerEntry* entry_for(LedgerFile* f, int pid, uint64_t now) {
  int n = f->n.load(std::memory_order_relaxed);
  LedgerEntry* free_e = nullptr;
  for (int i = 0; i < n; i++) {
    const int p = f->e[i].pid.load(std::memory_order_relaxed);
    if (p == pid) return &f->e[i];
    if (!p && !free_e) free_e = &f->e[i];
  }
  if (!free_e) {
    if (n >= kLedgerMaxPids) return nullptr;
    free_e = &f->e[n];
    f->n.store(n + 1, std::memory_order_release);
  }
  // A fresh entry: counters start at zero before the PID is published.
  free_e->occ.store(0, std::memory_order_relaxed);
  free_e->charged_ns.store(0, std::memory_order_relaxed);
  free_e->busy_ns.store(0, std::memory_order_relaxed);
  free_e->seen_ns.store(now, std::memory_order_relaxed);
  free_e->pid.store(pid, std::memory_order_release);
  return free_e;
}

// One sample of one GPU: n occupancy reads, one consistent split of the interval.
int sample(Gpu& g, uint64_t now) {
  LedgerFile* f = g.f;
  const int64_t dt = g.last_ns ? (int64_t)std::min<uint64_t>(now - g.last_ns, 1'000'000'000ull) : 0;
  g.last_ns = now;
  std::vector<int64_t> occ(g.pids.size());
  int64_t total = 0;
  for (size_t i = 0; i < g.pids.size(); i++) {
    occ[i] = std::max<int64_t>(0, kfd_cu_occupancy(g.pids[i], g.gpu_id));
    total += occ[i];
  }
  std::map<int, int64_t> ppm;
  for (size_t i = 0; i < g.pids.size(); i++) {
    const int pid = g.pids[i];
    LedgerEntry* e = entry_for(f, pid, now);
    if (!e) continue;
    const int64_t share = total > 0 ? occ[i] * 1'000'000 / total : 0;
    auto it = g.prev_ppm.find(pid);
    const int64_t prev = it == g.prev_ppm.end() ? 0 : it->second;
    // Trapezoid over the interval between the two snapshots.
    if (dt > 0 && (prev || share)) e->charged_ns.fetch_add((uint64_t)(dt * (prev + share) / 2'000'000), std::memory_order_relaxed);
    e->occ.store((int32_t)occ[i], std::memory_order_relaxed);
    if (occ[i] > 0) e->busy_ns.store(now, std::memory_order_relaxed);
    ppm[pid] = share;
    g.gone_since.erase(pid);
  }
  g.prev_ppm.swap(ppm);
  // Entries of PIDs that left: occupancy 0 at once, reused after kForgetNs.
  const int n = f->n.load(std::memory_order_relaxed);
  for (int i = 0; i < n; i++) {
    const int p = f->e[i].pid.load(std::memory_order_relaxed);
    if (!p || std::find(g.pids.begin(), g.pids.end(), p) != g.pids.end()) continue;
    f->e[i].occ.store(0, std::memory_order_relaxed);
    auto [it, fresh] = g.gone_since.emplace(p, now);
    if (!fresh && now - it->second > kForgetNs) {
      f->e[i].pid.store(0, std::memory_order_release);
      g.gone_since.erase(it);
    }
  }
  f->total_occ.store(total, std::memory_order_relaxed);
  f->reads.fetch_add(g.pids.size(), std::memory_order_relaxed);
  f->samples.fetch_add(1, std::memory_order_relaxed);
  f->heartbeat_ns.store(now, std::memory_order_release);
  return (int)g.pids.size();
}

long arg_long(int argc, char** argv, const char* name, long def) {
  for (int i = 1; i + 1 < argc; i++)
    if (!strcmp(argv[i], name)) return strtol(argv[i + 1], nullptr, 10);
  return def;
}

const char* arg_str(int argc, char** argv, const char* name) {
  for (int i = 1; i + 1 < argc; i++)
    if (!strcmp(argv[i], name)) return argv[i + 1];
  return nullptr;
}

// One GPU's sampling loop (its own period and read budget).
void gpu_loop(Gpu* g, int64_t base_ns, int budget, long max_samples) {
  long rounds = 0;
  while (!g_stop && !g->stop.load(std::memory_order_relaxed)) {
    {
      std::lock_guard<std::mutex> l(g->mu);
      g->pids = g->next_pids;
    }
    const int64_t reads = sample(*g, now_ns());
    const int64_t period = sample_period_ns(base_ns, reads, budget, std::max<int64_t>(10'000'000, base_ns));
    g->f->period_ns.store((uint64_t)period, std::memory_order_relaxed);
    if (max_samples && ++rounds >= max_samples) break;
    struct timespec ts = {(time_t)(period / 1000000000), (long)(period % 1000000000)};
    nanosleep(&ts, nullptr);
  }
}

}  // namespace

int main(int argc, char** argv) {
  const char* dir = arg_str(argc, argv, "--dir");
  if (!dir) {
    fprintf(stderr, "usage: vgpu-ledger --dir <board dir> [--period-us 1000] [--read-budget 32] [--samples N] "
                    "[--gpu ID]...\n");
    return 2;
  }
  const int64_t base_ns = std::max(100L, arg_long(argc, argv, "--period-us", 1000)) * 1000;
  const int budget = (int)arg_long(argc, argv, "--read-budget", 32);
  const long max_samples = arg_long(argc, argv, "--samples", 0);  // tests: each GPU stops after N rounds
  if (const char* k = getenv("VGPU_KFD_ROOT")) g_kfd_proc_root = k;
  prctl(PR_SET_PDEATHSIG, SIGTERM);
  const pid_t parent = getppid();
  signal(SIGTERM, on_signal);
  signal(SIGINT, on_signal);

  std::set<uint32_t> always;
  for (int i = 1; i + 1 < argc; i++)
    if (!strcmp(argv[i], "--gpu")) always.insert((uint32_t)strtoul(argv[i + 1], nullptr, 10));
  Board board;
  board.open_readonly(dir);
  std::map<uint32_t, std::unique_ptr<Gpu>> gpus;
  auto retire = [](std::unique_ptr<Gpu>& g) {
    g->stop.store(true);
    if (g->th.joinable()) g->th.join();
    munmap(g->f, sizeof(LedgerFile));
  };
  // The board thread (this one): which GPUs hold limited containers, and their processes.
  while (!g_stop && getppid() == parent) {
    const uint64_t now = now_ns();
    std::set<uint32_t> active = always;
    for (const BoardPeer& p : board.refresh(now))
      for (uint32_t id : p.gpu_ids)
        if (id) active.insert(id);
    for (uint32_t id : active) {
      std::unique_ptr<Gpu>& g = gpus[id];
      if (!g) {
        g.reset(new Gpu());
        g->gpu_id = id;
        g->f = create_ledger(dir, id);
        if (!g->f) {
          fprintf(stderr, "vgpu-ledger: cannot create %s\n", ledger_path(dir, id).c_str());
          gpus.erase(id);
          continue;
        }
        g->next_pids = kfd_pids_on_gpu(id);
        g->th = std::thread(gpu_loop, g.get(), base_ns, budget, max_samples);
        continue;
      }
      std::vector<int> pids = kfd_pids_on_gpu(id);
      std::lock_guard<std::mutex> l(g->mu);
      g->next_pids.swap(pids);
    }
    // A GPU no container holds any more is no longer sampled (its ledger goes stale).
    for (auto it = gpus.begin(); it != gpus.end();) {
      if (active.count(it->first)) {
        ++it;
      } else {
        retire(it->second);
        it = gpus.erase(it);
      }
    }
    if (max_samples) {  // tests: done once every GPU thread has taken its samples
      bool all_done = !gpus.empty();
      for (auto& kv : gpus)
        all_done = all_done && kv.second->f->samples.load(std::memory_order_relaxed) >= (uint64_t)max_samples;
      if (all_done) break;
    }
    struct timespec ts = {0, 100'000'000};
    nanosleep(&ts, nullptr);
  }
  g_stop = 1;
  for (auto& kv : gpus) retire(kv.second);
  return 0;
}
