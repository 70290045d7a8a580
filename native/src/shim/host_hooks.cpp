// Pinned host memory: hipHostMalloc / hipHostAlloc / hipMallocHost / hipMemAllocHost and
// hipHostRegister, accounted against the container's VGPU_HOST_MEMORY_LIMIT.
//
// Reference: cuMemAllocHost_v2, cuMemHostAlloc and cuMemHostRegister_v2 are suspend-gated
// and OOM-checked (class (b) in SURVEY.md §2.3, [memory.c]). Page-locked RAM is a
// node-wide resource (the host-spill pool of oversubscribed vGPUs draws on the same RAM),
// so here it has a budget of its own in the container's region: admitted with the same
// CAS loop and dead-process reclaim as device memory, released on free / unregister, and
// dropped with the slot when a process exits. The allocations reach ROCr through the CPU
// pools, which the device-memory hooks (hsa_hooks.cpp) leave alone.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <mutex>

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"
#include "vgpu/region.h"

using namespace vgpu;

namespace {

using AllocFn3 = hipError_t (*)(void**, size_t, unsigned int);
using AllocFn2 = hipError_t (*)(void**, size_t);
using FreeFn = hipError_t (*)(void*);
using RegisterFn = hipError_t (*)(void*, size_t, unsigned int);

bool charge_host(size_t size) {
  ShimState& s = shim();
  if (s.region.charge_host(s.slot, size) == Charge::kOk) return true;
  VLOG_WARN("host memory OOM: request %zu bytes, pinned %lu of limit %lu", size, (unsigned long)s.region.host_usage(),
            (unsigned long)s.region.host_limit());
  return false;
}

void record(void* p, size_t size) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  s.host[reinterpret_cast<uintptr_t>(p)] = size;
}

}  // namespace

namespace vgpu {

void release_host(void* p) {
  ShimState& s = shim();
  if (!p || !s.active) return;
  uint64_t size = 0;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    auto it = s.host.find(reinterpret_cast<uintptr_t>(p));
    if (it == s.host.end()) return;
    size = it->second;
    s.host.erase(it);
  }
  if (s.slot >= 0 && !s.exiting.load()) s.region.uncharge_host(s.slot, size);
}

}  // namespace vgpu

namespace {

// Admission around the runtime's allocation. The first HIP call of a process initialises
// the runtime (and the shim, from the hsa_init hook) inside the real call, so a process
// whose first call this is is charged afterwards, and refused by releasing the memory.
template <typename Call, typename Undo>
hipError_t admit(void* const* out, size_t size, Call call, Undo undo) {
  ShimState& s = shim();
  gate_suspend();
  const bool pre = s.active && size;
  if (pre && !charge_host(size)) return hipErrorOutOfMemory;
  hipError_t e = call();
  void* p = out ? *out : nullptr;
  if (e != hipSuccess || !p) {
    if (pre) s.region.uncharge_host(s.slot, size);
    return e;
  }
  if (!pre) {
    if (!s.active || !size) return e;
    if (!charge_host(size)) {
      (void)undo(p);
      return hipErrorOutOfMemory;
    }
  }
  record(p, size);
  return e;
}

hipError_t host_free(void* p) {
  VGPU_REAL_AS(hipHostFree, FreeFn, "libamdhip64", nullptr);
  return real_hipHostFree ? real_hipHostFree(p) : hipErrorNotSupported;
}

}  // namespace

#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wdeprecated-declarations"

extern "C" {

hipError_t hipHostMalloc(void** ptr, size_t size, unsigned int flags) {
  VGPU_REAL_AS(hipHostMalloc, AllocFn3, "libamdhip64", nullptr);
  if (!real_hipHostMalloc) return hipErrorNotSupported;
  return admit(ptr, size, [&] { return real_hipHostMalloc(ptr, size, flags); }, host_free);
}

hipError_t hipHostAlloc(void** ptr, size_t size, unsigned int flags) {
  VGPU_REAL_AS(hipHostAlloc, AllocFn3, "libamdhip64", nullptr);
  if (!real_hipHostAlloc) return hipErrorNotSupported;
  return admit(ptr, size, [&] { return real_hipHostAlloc(ptr, size, flags); }, host_free);
}

hipError_t hipMallocHost(void** ptr, size_t size) {
  VGPU_REAL_AS(hipMallocHost, AllocFn2, "libamdhip64", nullptr);
  if (!real_hipMallocHost) return hipErrorNotSupported;
  return admit(ptr, size, [&] { return real_hipMallocHost(ptr, size); }, host_free);
}

hipError_t hipMemAllocHost(void** ptr, size_t size) {
  VGPU_REAL_AS(hipMemAllocHost, AllocFn2, "libamdhip64", nullptr);
  if (!real_hipMemAllocHost) return hipErrorNotSupported;
  return admit(ptr, size, [&] { return real_hipMemAllocHost(ptr, size); }, host_free);
}

hipError_t hipHostFree(void* ptr) {
  VGPU_REAL_AS(hipHostFree, FreeFn, "libamdhip64", nullptr);
  if (!real_hipHostFree) return hipErrorNotSupported;
  gate_suspend();
  // Released only once the runtime has let go of the memory: a failed free leaves it
  // pinned, and so charged (as hipHostUnregister below).
  hipError_t e = real_hipHostFree(ptr);
  if (e == hipSuccess) release_host(ptr);
  return e;
}

hipError_t hipFreeHost(void* ptr) {
  VGPU_REAL_AS(hipFreeHost, FreeFn, "libamdhip64", nullptr);
  if (!real_hipFreeHost) return hipErrorNotSupported;
  gate_suspend();
  // Released only once the runtime has let go of the memory: a failed free leaves it
  // pinned, and so charged (as hipHostUnregister below).
  hipError_t e = real_hipFreeHost(ptr);
  if (e == hipSuccess) release_host(ptr);
  return e;
}

hipError_t hipHostRegister(void* host_ptr, size_t size, unsigned int flags) {
  VGPU_REAL_AS(hipHostRegister, RegisterFn, "libamdhip64", nullptr);
  VGPU_REAL_AS(hipHostUnregister, FreeFn, "libamdhip64", nullptr);
  if (!real_hipHostRegister) return hipErrorNotSupported;
  void* p = host_ptr;
  return admit(&p, size, [&] { return real_hipHostRegister(host_ptr, size, flags); },
               [&](void* q) {
                 if (real_hipHostUnregister) (void)real_hipHostUnregister(q);
               });
}

hipError_t hipHostUnregister(void* host_ptr) {
  VGPU_REAL_AS(hipHostUnregister, FreeFn, "libamdhip64", nullptr);
  if (!real_hipHostUnregister) return hipErrorNotSupported;
  gate_suspend();
  hipError_t e = real_hipHostUnregister(host_ptr);
  if (e == hipSuccess) release_host(host_ptr);
  return e;
}

}  // extern "C"

#pragma GCC diagnostic pop
