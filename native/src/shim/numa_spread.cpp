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
// Nothing is narrowed when the allowed CPUs are already within the node (an exclusive cpuset
// from the kubelet's CPU manager, say), or do not meet it. A tenant opts out with
// VGPU_CPU_SPREAD=0: this is a placement hint, not a limit.
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
  const std::string path = std::string(root && *root ? root : "/sys") + "/devices/system/node/node" +
                           std::to_string(n) + "/cpulist";
  FILE* f = fopen(path.c_str(), "re");
  if (!f) return;
  char buf[4096] = {0};
  const size_t got = fread(buf, 1, sizeof(buf) - 1, f);
  fclose(f);
  buf[got] = 0;
  cpu_set_t want, allowed, both;
  if (!parse_cpulist(buf, &want) || sched_getaffinity(0, sizeof(allowed), &allowed) != 0) return;
  CPU_AND(&both, &want, &allowed);
  const int nb = CPU_COUNT(&both), na = CPU_COUNT(&allowed);
  if (nb == 0 || nb == na) return;   // no overlap, or already within the node
  if (sched_setaffinity(0, sizeof(both), &both) == 0)
    VLOG_INFO("CPU affinity narrowed to NUMA node %ld: %d of %d allowed CPUs (--numa-spread)", n, nb, na);
}

}  // namespace
}  // namespace vgpu
