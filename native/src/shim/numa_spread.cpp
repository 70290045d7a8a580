// CPU placement of a vGPU's processes (--numa-spread, VGPU_CPU_NODE).
//
// Two launch-bound PyTorch processes of one MI355X whose threads run on the same CPU socket
// are no faster together than one alone: LSTM inference pairs 1.00x, ResNet-152 b=10 pairs
// 1.00x. The same pairs with one process per socket run at 2.0x and 1.55x. A lone process runs
// equally fast from either socket (profiles/r5d). The effect is per socket, not per L3 domain
// or SMT core. Where the host memory lives does not matter. The C++ empty-kernel launch path
// alone does not show it.
//
// The plugin therefore gives vGPU k of a GPU a CPU node (the GPU's own first, then the
// others, round robin: plugin/vdevice.py::assign_cpu_nodes). Here, before the program's main()
// - while its only thread is the one that runs the constructors - the process's CPU affinity
// is narrowed to that node's CPUs. Threads and processes it creates later inherit it.
//
// It is a placement within the shared pool, never a cut of CPUs the pod was granted. Nothing is
// narrowed when
// * the allowed CPUs are already within the node, or do not meet it;
// * they are the container's own: the kubelet's CPU manager (static policy) gives a Guaranteed
//   pod with an integer CPU request an exclusive cpuset of exactly that many CPUs, so a CPU
//   quota (cgroup cpu.max, or cpu.cfs_quota_us / cpu.cfs_period_us) equal to the allowed
//   count marks an exclusive set - kept whole even when it spans both sockets;
// * the node's share of the allowed CPUs is smaller than the container's CPU quota (it would
//   throttle a CPU-heavy tenant - DataLoader workers, tokenizers - below what it pays for).
// A tenant opts out with VGPU_CPU_SPREAD=0: this is a placement hint, not a limit.
#include <sched.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>

#include "vgpu/log.h"

namespace vgpu {
namespace {

bool parse_cpulist(const char* s, cpu_set_t* out) {
  CPU_ZERO(out);
  bool any = false;
  while (*s) {
    char* end = nullptr;
    long lo = strtol(s, &end, 10);
    if (end == s) break;
    long hi = lo;
    s = end;
    if (*s == '-') {
      hi = strtol(s + 1, &end, 10);
      s = end;
    }
    for (long c = lo; c <= hi && c < CPU_SETSIZE; c++)
      if (c >= 0) {
        CPU_SET((int)c, out);
        any = true;
      }
    while (*s == ',' || *s == '\n' || *s == ' ') s++;
  }
  return any;
}

bool read_small(const std::string& path, char* buf, size_t n) {
  FILE* f = fopen(path.c_str(), "re");
  if (!f) return false;
  const size_t got = fread(buf, 1, n - 1, f);
  fclose(f);
  buf[got] = 0;
  return got > 0;
}

// The container's CPU quota in CPUs (rounded up), or -1 when it has none (unlimited, or no
// cgroup file readable). `fs` is the cgroup mount (/sys/fs/cgroup). Inside a container the
// cgroup namespace makes its own cgroup the root; otherwise /proc/self/cgroup names it.
long cpu_quota_cpus(const std::string& fs) {
  char buf[256];
  std::string rel;
  if (FILE* f = fopen("/proc/self/cgroup", "re")) {
    char line[1024];
    while (fgets(line, sizeof(line), f))
      if (strncmp(line, "0::", 3) == 0) {
        rel = line + 3;
        while (!rel.empty() && (rel.back() == '\n' || rel.back() == '/')) rel.pop_back();
      }
    fclose(f);
  }
  long long quota = -1, period = 0;
  for (const std::string& dir : {fs + rel, fs}) {   // cgroup v2
    if (!read_small(dir + "/cpu.max", buf, sizeof(buf))) continue;
    if (strncmp(buf, "max", 3) == 0) return -1;
    if (sscanf(buf, "%lld %lld", &quota, &period) == 2 && quota > 0 && period > 0) return (long)((quota + period - 1) / period);
    return -1;
  }
  for (const char* ctl : {"/cpu,cpuacct", "/cpu"}) {  // cgroup v1
    char p[64];
    if (!read_small(fs + ctl + "/cpu.cfs_quota_us", buf, sizeof(buf))) continue;
    quota = atoll(buf);
    if (!read_small(fs + ctl + "/cpu.cfs_period_us", p, sizeof(p))) return -1;
    period = atoll(p);
    return quota > 0 && period > 0 ? (long)((quota + period - 1) / period) : -1;
  }
  return -1;
}

__attribute__((constructor)) void numa_spread_ctor() {
  const char* node = getenv("VGPU_CPU_NODE");
  if (!node || !*node) return;
  const char* opt = getenv("VGPU_CPU_SPREAD");
  if (opt && *opt == '0') return;
  char* end = nullptr;
  const long n = strtol(node, &end, 10);
  if (end == node || n < 0) return;
  log_init_from_env();
  const char* root = getenv("VGPU_SYSFS_ROOT");   // tests: a fake sysfs tree
  const std::string sys = root && *root ? root : "/sys";
  char buf[4096] = {0};
  if (!read_small(sys + "/devices/system/node/node" + std::to_string(n) + "/cpulist", buf, sizeof(buf))) return;
  cpu_set_t want, allowed, both;
  if (!parse_cpulist(buf, &want) || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  CPU_AND(&both, &want, &allowed);
  const int nb = CPU_COUNT(&both), na = CPU_COUNT(&allowed);
  if (nb == 0 || nb == na) return;   // no overlap, or already within the node
  const long quota = cpu_quota_cpus(sys + "/fs/cgroup");
  if (quota == na) {
    VLOG_INFO("CPU affinity kept: %d CPUs = the container's CPU quota (an exclusive cpuset)", na);
    return;
  }
  if (quota > nb) {
    VLOG_INFO("CPU affinity kept: NUMA node %ld holds %d of the allowed CPUs, below the quota of %ld", n, nb, quota);
    return;
  }
  if (sched_setaffinity(0, sizeof(both), &both) == 0)
    VLOG_INFO("CPU affinity narrowed to NUMA node %ld: %d of %d allowed CPUs (--numa-spread)", n, nb, na);
}

}  // namespace
}  // namespace vgpu
