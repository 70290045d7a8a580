// In-process control API exported by the shim (reference-name mapping):
//   suspend_all / resume_all                → vgpu_suspend_all / vgpu_resume_all
//   set_current_device_memory_limit         → vgpu_set_current_device_memory_limit
//   set_current_device_sm_limit_scale       → vgpu_set_current_device_cu_limit
//   get_current_device_{memory_limit,usage} → vgpu_get_current_device_*
//   cuVGPUViewAllocator (debug dump)        → vgpu_view_allocator
// Names are prefixed: the shim is preloaded into arbitrary programs and must not
// collide with their symbols.

// hip_runtime_api.h must be told its platform when a host compiler (g++) includes it;
// AMD is the only platform this code is built for.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <cstdio>

#include "real.h"
#include "shim.h"

using namespace vgpu;

namespace {
int current_device() { return current_hip_agent(); }
bool ok() { return shim_attach_region_only(); }
}  // namespace

extern "C" {

__attribute__((visibility("default"))) int vgpu_suspend_all() {
  if (!ok()) return -1;
  shim().region.suspend_all();
  return 0;
}

__attribute__((visibility("default"))) int vgpu_resume_all() {
  if (!ok()) return -1;
  shim().region.resume_all();
  return 0;
}

// The in-container setters may only lower a limit (the reference's raise it: an in-container
// escape, [multiprocess_memory_limit.c:806-808]); raising is the operator's, from the node
// (vgpuctl / the monitor, which write the region directly).
__attribute__((visibility("default"))) int vgpu_set_current_device_memory_limit(uint64_t bytes) {
  if (!ok()) return -1;
  const int dev = current_device();
  const uint64_t cur = shim().region.limit(dev);
  if (!bytes || (cur && bytes > cur)) return -1;
  shim().region.set_limit(dev, bytes);
  return 0;
}

__attribute__((visibility("default"))) uint64_t vgpu_get_current_device_memory_limit() {
  return ok() ? shim().region.limit(current_device()) : 0;
}

__attribute__((visibility("default"))) uint64_t vgpu_get_current_device_memory_usage() {
  return ok() ? shim().region.usage(current_device()) : 0;
}

// Bytes of the current device's quota this process's container holds in host memory (virtual
// device memory, spill.cpp): falls as spills are promoted into HBM.
__attribute__((visibility("default"))) uint64_t vgpu_get_current_device_spilled() {
  return ok() ? shim().region.raw()->dev[current_device()].spilled.load() : 0;
}

// HBM of the current device holding shared virtual memory - this container's promoted spills
// and prefetched ranges, and (node board) other containers' - that ROCr's free-memory figure
// does not show; the shim takes it off the free HBM it reports and places by (spill.cpp).
__attribute__((visibility("default"))) uint64_t vgpu_get_current_device_hidden_vram() {
  return ok() ? hidden_vram(current_device()) : 0;
}

// Pinned host memory the container holds (VGPU_HOST_MEMORY_LIMIT's budget, host_hooks.cpp).
__attribute__((visibility("default"))) uint64_t vgpu_get_host_memory_usage() {
  return ok() ? shim().region.host_usage() : 0;
}

__attribute__((visibility("default"))) int vgpu_set_current_device_cu_limit(int pct) {
  if (!ok() || pct <= 0 || pct >= 100) return -1;
  const int dev = current_device();
  const int cur = shim().region.raw()->dev[dev].cu_limit_pct;
  if (cur > 0 && cur < 100 && pct > cur) return -1;
  shim().region.set_cu_limit(dev, pct);
  return 0;
}

__attribute__((visibility("default"))) int vgpu_get_current_device_cu_limit() {
  return ok() ? shim().region.raw()->dev[current_device()].cu_limit_pct : -1;
}

__attribute__((visibility("default"))) int vgpu_shim_active() { return shim().active ? 1 : 0; }

__attribute__((visibility("default"))) void vgpu_view_allocator() {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  fprintf(stderr, "[vGPU] allocator: %zu live allocations, %zu vmem handles, %zu SVM spills, slot %d\n",
          s.allocs.size(), s.vmem.size(), s.svm.size(), s.slot);
  for (const auto& kv : s.allocs)
    fprintf(stderr, "  %p size=%lu dev=%d kind=%d\n", (void*)kv.first, (unsigned long)kv.second.size, kv.second.dev,
            kv.second.kind);
  for (const auto& kv : s.svm)
    fprintf(stderr, "  %p size=%lu dev=%d svm %s\n", (void*)kv.first, (unsigned long)kv.second.size, kv.second.dev,
            kv.second.in_hbm ? "in HBM" : "in host memory");
}

}  // extern "C"
