// HIP-level interposition: kernel-launch and copy gates.
//
// Reference: cuLaunchKernel / cuLaunchCooperativeKernel [src/cuda/memory.c:598-611]
// run the suspend gate (wait_status_self) and the token-bucket rate_limiter before
// the real launch, and 41 copy/alloc hooks run the suspend gate. cuGraphLaunch is a
// plain passthrough there [graph.c:224-225], so graph replays escape the throttle;
// here a graph launch passes the same gates as a kernel launch, and the GPU-time limiter
// charges whatever its kernels run (ratelimit.h).
//
// Hot-path budget: a launch pays one predictable branch on process-local state, a
// relaxed increment of its own slot's launch counter, and relaxed loads of region words
// (generation, suspend flags, launch block, and in temporal mode the device's credit).
// The device lookup (hipGetDevice) only happens with several agents in temporal mode.

// hip_runtime_api.h must be told its platform when a host compiler (g++) includes it;
// AMD is the only platform this code is built for.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <mutex>
#include <unordered_map>
#include <vector>

#include "vgpu/region.h"

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

using namespace vgpu;

// hip_ext.h needs the HIP compiler; declare the one entry point we need from it.
extern "C" hipError_t hipExtModuleLaunchKernel(hipFunction_t f, uint32_t globalWorkSizeX, uint32_t globalWorkSizeY,
                                               uint32_t globalWorkSizeZ, uint32_t localWorkSizeX,
                                               uint32_t localWorkSizeY, uint32_t localWorkSizeZ,
                                               size_t sharedMemBytes, hipStream_t hStream, void** kernelParams,
                                               void** extra, hipEvent_t startEvent, hipEvent_t stopEvent,
                                               uint32_t flags);

using LaunchKernelFn = hipError_t (*)(const void*, dim3, dim3, void**, size_t, hipStream_t);
using CoopKernelFn = hipError_t (*)(const void*, dim3, dim3, void**, unsigned int, hipStream_t);
using MallocManagedFn = hipError_t (*)(void**, size_t, unsigned int);
using MallocAsyncFn = hipError_t (*)(void**, size_t, hipStream_t);
using MallocFromPoolAsyncFn = hipError_t (*)(void**, size_t, hipMemPool_t, hipStream_t);
using ExtLaunchKernelFn = hipError_t (*)(const void*, dim3, dim3, void**, size_t, hipStream_t, hipEvent_t, hipEvent_t,
                                         int);

namespace {

// VGPU_HOOK_LAUNCH=0: launch hooks become pure pass-throughs (diagnostics; disables the
// suspend gate, the launch block and the temporal limiter at launch). Read once at load.
bool g_launch_hooks_on = true;
__attribute__((constructor)) void launch_hook_ctor() {
  const char* s = getenv("VGPU_HOOK_LAUNCH");
  if (s && *s == '0') g_launch_hooks_on = false;
}

inline void launch_gate() {
  VGPU_STAT(kStatLaunch);
  if (__builtin_expect(!g_launch_hooks_on, 0)) return;
  ShimState& s = shim();
  if (__builtin_expect(!s.active, 1)) return;
  // Fast path: count (process-local; the maintenance thread publishes it), then three
  // relaxed loads of region words that only a controller writes.
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

int hip_device_agent(int hipdev) {
  ShimState& s = shim();
  if (s.n_agents <= 1 || hipdev < 0 || !s.region.attached()) return 0;
  static std::once_flag once;
  static int map[kMaxDevices];
  std::call_once(once, [&s] {
    for (int i = 0; i < kMaxDevices; i++) map[i] = i;
    VGPU_REAL_HIP(hipGetDeviceCount);
    VGPU_REAL_HIP(hipDeviceGetAttribute);
    int count = 0;
    if (!real_hipGetDeviceCount || !real_hipDeviceGetAttribute || real_hipGetDeviceCount(&count) != hipSuccess)
      return;
    const Region* r = s.region.raw();
    int found[kMaxDevices];
    for (int h = 0; h < count && h < kMaxDevices; h++) {
      int bus = -1, dev = -1, dom = -1;
      if (real_hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, h) != hipSuccess ||
          real_hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, h) != hipSuccess ||
          real_hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, h) != hipSuccess)
        return;
      int match = -1, n = 0;
      for (int a = 0; a < s.n_agents; a++) {
        const DeviceState& d = r->dev[a];
        if ((d.bdf >> 3) == ((uint32_t)bus << 5 | (uint32_t)dev) && d.domain == (uint32_t)dom) {
          match = a;
          n++;
        }
      }
      if (n != 1) return;  // unknown or shared address (compute partitions): keep the identity
      found[h] = match;
    }
    for (int h = 0; h < count && h < kMaxDevices; h++) map[h] = found[h];
    VLOG_DEBUG("HIP device -> agent map built for %d device(s)", count);
  });
  return hipdev < kMaxDevices && map[hipdev] < s.n_agents ? map[hipdev] : 0;
}

int current_hip_agent() {
  ShimState& s = shim();
  if (s.n_agents <= 1) return 0;
  VGPU_REAL_HIP(hipGetDevice);
  int d = 0;
  if (!real_hipGetDevice || real_hipGetDevice(&d) != hipSuccess) return 0;
  return hip_device_agent(d);
}

void gate_launch(int dev) {
  ShimState& s = shim();
  Region* r = s.region.raw();
  check_live_config();
  gate_suspend();
  if (dev < 0) {
    dev = 0;
    if (s.n_agents > 1) {
      bool any = false;
      for (int i = 0; i < s.n_agents; i++) any |= s.agents[i].temporal_active.load(std::memory_order_relaxed);
      if (any) dev = current_hip_agent();
    }
  }
  if (dev < 0 || dev >= s.n_agents) dev = 0;
  bool limited = s.agents[dev].temporal_active.load(std::memory_order_relaxed) &&
                 (r->hdr.utilization_switch.load(std::memory_order_relaxed) || config().cu_policy == CuPolicy::kForce);
  if (__builtin_expect(!limiter_would_block(r->hdr, r->dev[dev], limited), 1)) return;
  trace_push(limited ? "vgpu:throttle" : "vgpu:blocked");
  uint64_t waited = limiter_acquire(r->hdr, r->dev[dev], limited);
  trace_pop();
  if (waited && s.slot >= 0) r->procs[s.slot].throttle_ns.fetch_add(waited, std::memory_order_relaxed);
}

}  // namespace vgpu

extern "C" {

hipError_t hipLaunchKernel(const void* function_address, dim3 numBlocks, dim3 dimBlocks, void** args,
                           size_t sharedMemBytes, hipStream_t stream) {
  VGPU_REAL_HIP_T(hipLaunchKernel, LaunchKernelFn);
  launch_gate();
  return real_hipLaunchKernel(function_address, numBlocks, dimBlocks, args, sharedMemBytes, stream);
}

hipError_t hipExtLaunchKernel(const void* function_address, dim3 numBlocks, dim3 dimBlocks, void** args,
                              size_t sharedMemBytes, hipStream_t stream, hipEvent_t startEvent, hipEvent_t stopEvent,
                              int flags) {
  VGPU_REAL_HIP_T(hipExtLaunchKernel, ExtLaunchKernelFn);
  launch_gate();
  return real_hipExtLaunchKernel(function_address, numBlocks, dimBlocks, args, sharedMemBytes, stream, startEvent,
                                 stopEvent, flags);
}

hipError_t hipModuleLaunchKernel(hipFunction_t f, unsigned int gridDimX, unsigned int gridDimY, unsigned int gridDimZ,
                                 unsigned int blockDimX, unsigned int blockDimY, unsigned int blockDimZ,
                                 unsigned int sharedMemBytes, hipStream_t stream, void** kernelParams, void** extra) {
  VGPU_REAL_HIP(hipModuleLaunchKernel);
  launch_gate();
  return real_hipModuleLaunchKernel(f, gridDimX, gridDimY, gridDimZ, blockDimX, blockDimY, blockDimZ, sharedMemBytes,
                                    stream, kernelParams, extra);
}

hipError_t hipExtModuleLaunchKernel(hipFunction_t f, uint32_t globalWorkSizeX, uint32_t globalWorkSizeY,
                                    uint32_t globalWorkSizeZ, uint32_t localWorkSizeX, uint32_t localWorkSizeY,
                                    uint32_t localWorkSizeZ, size_t sharedMemBytes, hipStream_t hStream,
                                    void** kernelParams, void** extra, hipEvent_t startEvent, hipEvent_t stopEvent,
                                    uint32_t flags) {
  VGPU_REAL_HIP(hipExtModuleLaunchKernel);
  launch_gate();
  return real_hipExtModuleLaunchKernel(f, globalWorkSizeX, globalWorkSizeY, globalWorkSizeZ, localWorkSizeX,
                                       localWorkSizeY, localWorkSizeZ, sharedMemBytes, hStream, kernelParams, extra,
                                       startEvent, stopEvent, flags);
}

hipError_t hipLaunchCooperativeKernel(const void* f, dim3 gridDim, dim3 blockDimX, void** kernelParams,
                                      unsigned int sharedMemBytes, hipStream_t stream) {
  VGPU_REAL_HIP_T(hipLaunchCooperativeKernel, CoopKernelFn);
  launch_gate();
  return real_hipLaunchCooperativeKernel(f, gridDim, blockDimX, kernelParams, sharedMemBytes, stream);
}

hipError_t hipModuleLaunchCooperativeKernel(hipFunction_t f, unsigned int gridDimX, unsigned int gridDimY,
                                            unsigned int gridDimZ, unsigned int blockDimX, unsigned int blockDimY,
                                            unsigned int blockDimZ, unsigned int sharedMemBytes, hipStream_t stream,
                                            void** kernelParams) {
  VGPU_REAL_HIP(hipModuleLaunchCooperativeKernel);
  launch_gate();
  return real_hipModuleLaunchCooperativeKernel(f, gridDimX, gridDimY, gridDimZ, blockDimX, blockDimY, blockDimZ,
                                               sharedMemBytes, stream, kernelParams);
}

hipError_t hipGraphLaunch(hipGraphExec_t graphExec, hipStream_t stream) {
  VGPU_REAL_HIP(hipGraphLaunch);
  VGPU_STAT(kStatGraphLaunch);
  // A graph replay is one launch for the gates: the temporal limiter charges GPU time,
  // not launches, so a graph costs what its kernels run (the reference's cuGraphLaunch
  // bypassed the throttle entirely, [graph.c:224-225]).
  launch_gate();
  return real_hipGraphLaunch(graphExec, stream);
}

// Managed memory (reference: cuMemAllocManaged is an accounted allocation, class (a) in
// SURVEY.md §2.3). Depending on XNACK/HMM mode CLR may back it with system memory that
// never reaches the HSA pool hooks, so it is charged here unless the pool hook already
// charged the same pointer; past the quota the allocation is released and refused.
hipError_t hipMallocManaged(void** dev_ptr, size_t size, unsigned int flags) {
  VGPU_REAL_HIP_T(hipMallocManaged, MallocManagedFn);
  VGPU_REAL_HIP(hipFree);
  ShimState& s = shim();
  gate_suspend();
  // The first HIP call of a process initialises the runtime (and the shim, from the
  // hsa_init hook) inside the real call, so `active` is only meaningful afterwards:
  // charge after the allocation and release it again when over the quota.
  hipError_t e = real_hipMallocManaged(dev_ptr, size, flags);
  if (!s.active || size == 0 || e != hipSuccess || !dev_ptr || !*dev_ptr) return e;
  uintptr_t key = reinterpret_cast<uintptr_t>(*dev_ptr);
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    bool pooled = s.allocs.count(key) != 0;
    VLOG_DEBUG("hipMallocManaged(%zu) -> %p (%s)", size, *dev_ptr, pooled ? "charged by the pool hook" : "charging");
    if (pooled) return e;  // already charged by hsa_amd_memory_pool_allocate
  }
  const int dev = current_hip_agent();
  if (s.region.charge(s.slot, dev, size, kMemData) != Charge::kOk) {
    (void)real_hipFree(*dev_ptr);
    *dev_ptr = nullptr;
    return hipErrorOutOfMemory;
  }
  std::lock_guard<std::mutex> g(s.alloc_mu);
  s.managed[key] = AllocRec{size, dev, kMemData};
  return e;
}

// Stream-ordered allocations (hipMallocAsync / hipMallocFromPoolAsync) come from a HIP
// memory pool that grows through hsa_amd_vmem_handle_create in chunks; the quota is
// enforced there like for every other allocation. But when a chunk is refused, the HIP
// runtime of ROCm 7.x does not unwind the partly grown request and crashes (measured:
// hip_alloc_probe async segfaults right after the refused chunk, profiles/r1w). So such a
// request is admitted here, before the pool grows: it proceeds when the quota has room
// for all of it (plus one pool chunk of slack), or when the pool's cached free memory
// (reserved - used) can hold it; otherwise the caller gets hipErrorOutOfMemory, as for
// any refused allocation.
namespace {

constexpr uint64_t kPoolSlack = 64ull << 20;

bool async_admissible(hipMemPool_t pool, size_t size) {
  ShimState& s = shim();
  if (!s.active || size == 0) return true;
  int hipdev = 0;
  if (s.n_agents > 1) {
    VGPU_REAL_HIP(hipGetDevice);
    if (!real_hipGetDevice || real_hipGetDevice(&hipdev) != hipSuccess) hipdev = 0;
  }
  const int dev = hip_device_agent(hipdev);  // the region's device (agent) for the HIP device
  const uint64_t lim = s.region.limit(dev);
  if (!lim || config().oversubscribe) return true;
  if (s.region.usage(dev) + size + kPoolSlack <= lim) return true;
  if (!pool) {
    VGPU_REAL_HIP(hipDeviceGetMemPool);
    if (!real_hipDeviceGetMemPool || real_hipDeviceGetMemPool(&pool, hipdev) != hipSuccess) pool = nullptr;
  }
  if (pool) {
    VGPU_REAL_HIP(hipMemPoolGetAttribute);
    uint64_t reserved = 0, used = 0;
    if (real_hipMemPoolGetAttribute &&
        real_hipMemPoolGetAttribute(pool, hipMemPoolAttrReservedMemCurrent, &reserved) == hipSuccess &&
        real_hipMemPoolGetAttribute(pool, hipMemPoolAttrUsedMemCurrent, &used) == hipSuccess && reserved >= used &&
        size <= reserved - used)
      return true;  // served from memory the pool already holds (and the quota counts)
  }
  VLOG_WARN("device %d OOM (stream-ordered): request %zu bytes, usage %lu of limit %lu", dev, size,
            (unsigned long)s.region.usage(dev), (unsigned long)lim);
  return false;
}

}  // namespace

hipError_t hipMallocAsync(void** dev_ptr, size_t size, hipStream_t stream) {
  VGPU_REAL_HIP_T(hipMallocAsync, MallocAsyncFn);
  if (!real_hipMallocAsync) return hipErrorNotSupported;
  gate_suspend();
  if (!async_admissible(nullptr, size)) return hipErrorOutOfMemory;
  return real_hipMallocAsync(dev_ptr, size, stream);
}

hipError_t hipMallocFromPoolAsync(void** dev_ptr, size_t size, hipMemPool_t mem_pool, hipStream_t stream) {
  VGPU_REAL_HIP_T(hipMallocFromPoolAsync, MallocFromPoolAsyncFn);
  if (!real_hipMallocFromPoolAsync) return hipErrorNotSupported;
  gate_suspend();
  if (!async_admissible(mem_pool, size)) return hipErrorOutOfMemory;
  return real_hipMallocFromPoolAsync(dev_ptr, size, mem_pool, stream);
}

hipError_t hipFree(void* ptr) {
  VGPU_REAL_HIP(hipFree);
  ShimState& s = shim();
  if (__builtin_expect(s.active && ptr != nullptr, 1)) {
    AllocRec rec{0, -1, 0};
    {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      if (!s.managed.empty()) {
        auto it = s.managed.find(reinterpret_cast<uintptr_t>(ptr));
        if (it != s.managed.end()) {
          rec = it->second;
          s.managed.erase(it);
        }
      }
    }
    if (rec.dev >= 0 && s.slot >= 0 && !s.exiting.load()) s.region.uncharge(s.slot, rec.dev, rec.size, kMemData);
  }
  return real_hipFree(ptr);
}

// Copy/set gates (suspend only), mirroring the reference's wait_status_self set.
hipError_t hipMemcpy(void* dst, const void* src, size_t sizeBytes, hipMemcpyKind kind) {
  VGPU_REAL_HIP(hipMemcpy);
  VGPU_STAT(kStatCopy);
  gate_suspend();
  return real_hipMemcpy(dst, src, sizeBytes, kind);
}

hipError_t hipMemcpyAsync(void* dst, const void* src, size_t sizeBytes, hipMemcpyKind kind, hipStream_t stream) {
  VGPU_REAL_HIP(hipMemcpyAsync);
  VGPU_STAT(kStatCopy);
  gate_suspend();
  return real_hipMemcpyAsync(dst, src, sizeBytes, kind, stream);
}

hipError_t hipMemcpyWithStream(void* dst, const void* src, size_t sizeBytes, hipMemcpyKind kind, hipStream_t stream) {
  VGPU_REAL_HIP(hipMemcpyWithStream);
  VGPU_STAT(kStatCopy);
  gate_suspend();
  return real_hipMemcpyWithStream(dst, src, sizeBytes, kind, stream);
}

hipError_t hipMemcpyPeerAsync(void* dst, int dstDeviceId, const void* src, int srcDevice, size_t sizeBytes,
                              hipStream_t stream) {
  VGPU_REAL_HIP(hipMemcpyPeerAsync);
  VGPU_STAT(kStatCopy);
  gate_suspend();
  return real_hipMemcpyPeerAsync(dst, dstDeviceId, src, srcDevice, sizeBytes, stream);
}

hipError_t hipMemset(void* dst, int value, size_t sizeBytes) {
  VGPU_REAL_HIP(hipMemset);
  VGPU_STAT(kStatSet);
  gate_suspend();
  return real_hipMemset(dst, value, sizeBytes);
}

hipError_t hipMemsetAsync(void* dst, int value, size_t sizeBytes, hipStream_t stream) {
  VGPU_REAL_HIP(hipMemsetAsync);
  VGPU_STAT(kStatSet);
  gate_suspend();
  return real_hipMemsetAsync(dst, value, sizeBytes, stream);
}

hipError_t hipMemsetD32Async(hipDeviceptr_t dst, int value, size_t count, hipStream_t stream) {
  VGPU_REAL_HIP(hipMemsetD32Async);
  VGPU_STAT(kStatSet);
  gate_suspend();
  return real_hipMemsetD32Async(dst, value, count, stream);
}

}  // extern "C"
