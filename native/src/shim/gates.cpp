// Table-driven HIP gates and the routing of runtime symbol lookups back into the shim.
//
// Reference parity:
//   * cuLaunchKernel / cuLaunchCooperativeKernel run the suspend gate and the rate limiter
//     [memory.c:598-611]; 41 copy/set/IPC/pointer/advise hooks run the suspend gate
//     (wait_status_self). Here every launch, copy and set variant libamdhip64 exports is
//     gated (src/shim/hip_gates.def): the *_spt per-thread-stream forms, the *MultiDevice
//     forms, hipLaunchKernelExC / hipDrvLaunchKernelEx, hipHccModuleLaunchKernel,
//     hipLaunchByPtr and graph replays included.
//   * dlsym [libvgpu.c:109-124] and cuGetProcAddress(_v2) [cuda/hook.c:299-357] route
//     runtime lookups of hooked names back into the shim. Here hipGetProcAddress does the
//     same (hip_hook_for_real), and the dlsym/dlvsym interposers (dlsym_hook.cpp) redirect
//     lookups of hooked hip* names made on a libamdhip64 handle: Triton - and so every
//     torch.compile tenant - resolves hipGetProcAddress with dlsym and fetches its launch
//     entry points through it (triton/backends/amd/driver.py).
//
// The gates are generated assembly trampolines (native/tools/gen_hip_gates.py): they save
// the argument registers, call vgpu_gate_enter(index) and tail-jump to the real entry
// point it returns, so no prototype is involved and a new runtime's variant only needs a
// row in the table (tests/test_hip_gates.py compares the table with `nm -D`).
#include <dlfcn.h>

#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"
#include "vgpu/region.h"

using namespace vgpu;

namespace vgpu {
// VGPU_HOOK_LAUNCH=0: launch gates become pure pass-throughs (diagnostics; disables the
// suspend gate, the launch block and the temporal limiter at launch). Read once at load.
bool g_launch_hooks_on = true;
}  // namespace vgpu

namespace {

enum GateKind : int { k_launch, k_graph, k_copy, k_set, k_suspend, k_device, k_hook, k_host };

struct GateDef {
  const char* name;
  const char* version;
  GateKind kind;
  unsigned devargs;  // device rows: bit i = argument i+1 is a device ordinal
};

const GateDef kGates[] = {
#define VGPU_GATE(idx, kind, name, ver, mask) {#name, ver, k_##kind, mask},
#include "hip_gates.inc"
#undef VGPU_GATE
};
constexpr int kNumGates = sizeof(kGates) / sizeof(kGates[0]);

std::atomic<void*> g_real[kNumGates];  // the runtime's entry points (resolved on first use)
void* g_self[kNumGates];               // the shim's own definitions (routing)
std::once_flag g_all_once;

// VGPU_HOOK_PROCADDR=0: hipGetProcAddress and dlsym on libamdhip64 return the runtime's
// entry points unchanged (diagnostics: measures what the routing buys). Both switches are
// ignored in a container with the plugin's limits file: they would lift enforcement.
bool g_route_on = true;
__attribute__((constructor)) void gates_ctor() {
  if (ceiling_present()) return;
  const char* s = getenv("VGPU_HOOK_LAUNCH");
  if (s && *s == '0') g_launch_hooks_on = false;
  s = getenv("VGPU_HOOK_PROCADDR");
  if (s && *s == '0') g_route_on = false;
}

// hipErrorNotSupported, for an entry point this runtime does not have (every gated entry
// point returns hipError_t, so the value lands where the caller expects it).
int gate_unsupported() { return 801; }

void* real_of(int i) {
  void* p = g_real[i].load(std::memory_order_acquire);
  if (__builtin_expect(p != nullptr, 1)) return p;
  p = resolve_real("libamdhip64", kGates[i].name, kGates[i].version, /*quiet=*/true);
  if (!p) p = reinterpret_cast<void*>(&gate_unsupported);
  g_real[i].store(p, std::memory_order_release);
  return p;
}

// Resolves every entry of the table once: the runtime's definition and the shim's own.
void resolve_all() {
  std::call_once(g_all_once, [] {
    Dl_info self;
    void* h = nullptr;
    if (dladdr(reinterpret_cast<void*>(&resolve_all), &self) && self.dli_fname)
      h = dlopen(self.dli_fname, RTLD_NOLOAD | RTLD_LAZY);
    for (int i = 0; i < kNumGates; i++) {
      (void)real_of(i);
      g_self[i] = h ? real_dlvsym(h, kGates[i].name, kGates[i].version) : nullptr;
      if (g_self[i]) {
        Dl_info di;
        if (!dladdr(g_self[i], &di) || di.dli_fbase != self.dli_fbase) g_self[i] = nullptr;
      }
    }
    if (h) dlclose(h);
  });
}

inline void launch_gate() {
  if (__builtin_expect(!g_launch_hooks_on, 0)) return;
  ShimState& s = shim();
  if (__builtin_expect(!s.active, 1)) return;
  // Fast path: count (process-local; the maintenance thread publishes it), then relaxed
  // loads of region words that only a controller writes.
  s.launches.fetch_add(1, std::memory_order_relaxed);
  const Region* r = s.region.raw();
  if (__builtin_expect(r->hdr.generation.load(std::memory_order_relaxed) ==
                               s.seen_generation.load(std::memory_order_relaxed) &&
                           !gate_needed() && r->hdr.recent_kernel.load(std::memory_order_relaxed) >= 0 &&
                           !s.any_temporal.load(std::memory_order_relaxed),
                       1))
    return;
  gate_launch(-1);
}

}  // namespace

namespace vgpu {

void* hip_hook_for_real(const void* real) {
  if (!g_route_on || !real) return nullptr;
  resolve_all();
  for (int i = 0; i < kNumGates; i++)
    if (g_real[i].load(std::memory_order_relaxed) == real && g_self[i]) return g_self[i];
  return nullptr;
}

void* hip_hook_for_name(const char* name, const char* version, const void* real) {
  if (!g_route_on || !real) return nullptr;
  for (int i = 0; i < kNumGates; i++) {
    if (strcmp(kGates[i].name, name) != 0) continue;
    if (version && strcmp(kGates[i].version, version) != 0) return nullptr;
    resolve_all();
    // Only a lookup that found the very entry point the hook forwards to is redirected:
    // a second HIP runtime in the process (another libamdhip64) keeps its own functions.
    if (g_real[i].load(std::memory_order_relaxed) != real) {
      VLOG_WARN("%s resolved to %p in another HIP runtime than the gated one (%p); not routed", name, real,
                g_real[i].load(std::memory_order_relaxed));
      return nullptr;
    }
    return g_self[i];
  }
  return nullptr;
}

}  // namespace vgpu

extern "C" {

// Called by the generated trampolines (hip_gates.S) with the row index of the entry point
// and the saved argument registers (rdi rsi rdx rcx r8 r9, in order).
__attribute__((visibility("hidden"))) void* vgpu_gate_enter(int idx, uint64_t* regs) {
  switch (kGates[idx].kind) {
    case k_device:
      gate_suspend();
      if (__builtin_expect(vdev_split_active(), 0))
        for (int a = 0; a < 6; a++)
          if (kGates[idx].devargs & (1u << a)) regs[a] = (uint64_t)(uint32_t)vdev_to_phys((int)(uint32_t)regs[a]);
      break;
    case k_launch:
      VGPU_STAT(kStatLaunch);
      launch_gate();
      break;
    case k_graph:
      // A graph replay is one launch for the gates: the temporal limiter charges GPU time,
      // not launches, so a graph costs what its kernels run.
      VGPU_STAT(kStatGraphLaunch);
      launch_gate();
      break;
    case k_copy:
      VGPU_STAT(kStatCopy);
      gate_suspend();
      break;
    case k_set:
      VGPU_STAT(kStatSet);
      gate_suspend();
      break;
    default:
      gate_suspend();
      break;
  }
  return real_of(idx);
}

// hipGetProcAddress (hip_6.1): the runtime's answer, with the shim's hook substituted when
// the answer is an entry point the shim gates (including per-thread-stream and versioned
// variants the flags / version select: the match is by address).
__attribute__((visibility("default"))) int hipGetProcAddress(const char* symbol, void** pfn, int hip_version,
                                                             uint64_t flags, int* status) {
  using Fn = int (*)(const char*, void**, int, uint64_t, int*);
  static int self_idx = [] {
    for (int i = 0; i < kNumGates; i++)
      if (!strcmp(kGates[i].name, "hipGetProcAddress")) return i;
    return -1;
  }();
  void* r = self_idx >= 0 ? real_of(self_idx) : nullptr;
  if (!r || r == reinterpret_cast<void*>(&gate_unsupported)) return 801;
  int rc = reinterpret_cast<Fn>(r)(symbol, pfn, hip_version, flags, status);
  if (rc == 0 && pfn && *pfn) {
    if (void* h = hip_hook_for_real(*pfn)) {
      VLOG_DEBUG("hipGetProcAddress(%s): routed to the shim", symbol ? symbol : "?");
      *pfn = h;
    }
  }
  return rc;
}

}  // extern "C"
