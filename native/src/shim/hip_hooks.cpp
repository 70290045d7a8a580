// HIP-level interposition with semantics: the launch gate's slow path, the HIP device ->
// agent map, and the device allocations that do not (only) pass the HSA pool hooks.
//
// The launch / copy / set entry points themselves are generated trampolines (gates.cpp,
// hip_gates.def). Reference: cuLaunchKernel / cuLaunchCooperativeKernel
// [src/cuda/memory.c:598-611] run the suspend gate (wait_status_self) and the
// token-bucket rate_limiter before the real launch.
//
// Hot-path budget: a launch pays one predictable branch on process-local state, a
// relaxed increment of its own slot's launch counter, and relaxed loads of region words
// (generation, suspend flags, launch block, and in temporal mode the device's credit).
// The device lookup (hipGetDevice) only happens with several agents in temporal mode.

// hip_runtime_api.h must be told its platform when a host compiler (g++) includes it;
// AMD is the only platform this code is built for.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <strings.h>

#include <atomic>
#include <cstring>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "vgpu/region.h"

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

using namespace vgpu;

using MallocManagedFn = hipError_t (*)(void**, size_t, unsigned int);
using MallocAsyncFn = hipError_t (*)(void**, size_t, hipStream_t);
using MallocFromPoolAsyncFn = hipError_t (*)(void**, size_t, hipMemPool_t, hipStream_t);

namespace vgpu {

namespace {

// HIP device ordinal -> agent index as CLR derives it from HIP_VISIBLE_DEVICES
// (CUDA_VISIBLE_DEVICES when that is unset): each entry is an agent index or an agent
// UUID, and CLR stops at the first entry that names no device. Returns the number of
// entries, or -1 when neither variable is set (identity).
int visible_from_env(const ShimState& s, int* out) {
  const char* v = getenv("HIP_VISIBLE_DEVICES");
  if (!v) v = getenv("CUDA_VISIBLE_DEVICES");
  if (!v) return -1;
  const Region* r = s.region.raw();
  int n = 0;
  for (const char* p = v; *p && n < kMaxDevices;) {
    const char* e = p;
    while (*e && *e != ',') e++;
    std::string tok(p, (size_t)(e - p));
    int idx = -1;
    if (!tok.empty() && tok.find_first_not_of("0123456789") == std::string::npos) {
      idx = atoi(tok.c_str());
    } else {
      for (int a = 0; a < s.n_agents && idx < 0; a++)
        if (!strcasecmp(r->dev[a].uuid, tok.c_str())) idx = a;
    }
    if (idx < 0 || idx >= s.n_agents) break;
    out[n++] = idx;
    p = *e ? e + 1 : e;
  }
  return n;
}

// Builds the HIP device -> agent map: by PCI address where it is unique (robust to any
// reordering), by the visible-devices list where several agents share one address
// (compute partitions exposed as GPUs). False when the runtime cannot answer yet.
bool build_device_map(ShimState& s, int* map) {
  VGPU_REAL_HIP(hipGetDeviceCount);
  VGPU_REAL_HIP(hipDeviceGetAttribute);
  int count = 0;
  if (!real_hipGetDeviceCount || real_hipGetDeviceCount(&count) != hipSuccess || count <= 0) return false;
  int env[kMaxDevices];
  const int n_env = visible_from_env(s, env);
  const Region* r = s.region.raw();
  for (int h = 0; h < kMaxDevices; h++) map[h] = h < s.n_agents ? h : 0;
  for (int h = 0; h < count && h < kMaxDevices; h++) {
    int by_env = n_env < 0 ? h : (h < n_env ? env[h] : -1);
    int by_bdf = -1, bus = -1, dev = -1, dom = -1;
    if (real_hipDeviceGetAttribute && real_hipDeviceGetAttribute(&bus, hipDeviceAttributePciBusId, h) == hipSuccess &&
        real_hipDeviceGetAttribute(&dev, hipDeviceAttributePciDeviceId, h) == hipSuccess &&
        real_hipDeviceGetAttribute(&dom, hipDeviceAttributePciDomainId, h) == hipSuccess) {
      int n = 0;
      for (int a = 0; a < s.n_agents; a++) {
        const DeviceState& d = r->dev[a];
        if ((d.bdf >> 3) == ((uint32_t)bus << 5 | (uint32_t)dev) && d.domain == (uint32_t)dom) {
          by_bdf = a;
          n++;
        }
      }
      if (n != 1) by_bdf = -1;  // shared address (partitions) or unknown: the list decides
    }
    const int pick = by_bdf >= 0 ? by_bdf : by_env;
    if (pick < 0 || pick >= s.n_agents) return false;
    map[h] = pick;
  }
  VLOG_DEBUG("HIP device -> agent map built for %d device(s)", count);
  return true;
}

}  // namespace

int hip_device_agent(int hipdev) {
  ShimState& s = shim();
  if (s.n_agents <= 1 || hipdev < 0 || hipdev >= kMaxDevices || !s.region.attached()) return 0;
  static std::atomic<bool> built{false};
  static int map[kMaxDevices];
  static std::mutex mu;
  static uint64_t next_try = 0;
  if (__builtin_expect(!built.load(std::memory_order_acquire), 0)) {
    // Not cached on failure: a runtime that could not answer yet (or a transient error)
    // is asked again, at most every 100 ms, instead of pinning the process to a guess.
    std::lock_guard<std::mutex> g(mu);
    if (!built.load(std::memory_order_relaxed) && now_ns() >= next_try) {
      int m[kMaxDevices];
      if (build_device_map(s, m)) {
        memcpy(map, m, sizeof(map));
        built.store(true, std::memory_order_release);
      } else {
        next_try = now_ns() + 100'000'000ull;
      }
    }
    if (!built.load(std::memory_order_relaxed)) {
      int env[kMaxDevices];
      const int n_env = visible_from_env(s, env);
      const int guess = n_env < 0 ? hipdev : (hipdev < n_env ? env[hipdev] : 0);
      return guess < s.n_agents ? guess : 0;
    }
  }
  return map[hipdev] < s.n_agents ? map[hipdev] : 0;
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
  uint64_t waited = 0;
  if (__builtin_expect(limiter_would_block(r->hdr, r->dev[dev], limited), 0)) {
    trace_push(limited ? "vgpu:throttle" : "vgpu:blocked");
    waited = limiter_acquire(r->hdr, r->dev[dev], limited);
    trace_pop();
  }
  // Background class next to a better one: bounded work in flight (watcher.cpp preempt_tick).
  const int cap = limited ? r->dev[dev].depth_cap.load(std::memory_order_relaxed) : 0;
  if (__builtin_expect(cap > 0, 0)) waited += wait_queue_depth(dev, cap);
  if (waited && s.slot >= 0) r->procs[s.slot].throttle_ns.fetch_add(waited, std::memory_order_relaxed);
}

}  // namespace vgpu

extern "C" {

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
  t_managed_alloc = true;  // the runtime's SVM calls for it are part of this allocation (svm_hooks.cpp)
  hipError_t e = real_hipMallocManaged(dev_ptr, size, flags);
  t_managed_alloc = false;
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
  // Pinned host memory freed through hipFree is released in the ROCr free hook (hsa_hooks.cpp).
  return real_hipFree(ptr);
}

}  // extern "C"
