// Pinned host memory, accounted against the container's VGPU_HOST_MEMORY_LIMIT at the layer
// every path goes through: ROCr's CPU memory pools and its memory locks.
//
// Reference: cuMemAllocHost_v2, cuMemHostAlloc and cuMemHostRegister_v2 are suspend-gated
// and OOM-checked (class (b) in SURVEY.md §2.3, [memory.c]) - the lowest user-visible layer
// of the CUDA stack. On MI355X that layer is ROCr: hipHostMalloc / hipHostAlloc /
// hipMallocHost / hipMemAllocHost (and PyTorch's pin_memory) reach
// hsa_amd_memory_pool_allocate on a CPU pool, hipHostRegister reaches
// hsa_amd_memory_lock_to_pool, and a program that uses ROCr directly (ctypes, an HSA
// application) calls those or hsa_amd_memory_lock itself. Charging there counts every path
// exactly once, the runtime's own staging buffers included (pinned RAM is pinned RAM).
// Page-locked RAM is a node-wide resource (the host-spill pool of oversubscribed vGPUs draws
// on the same RAM), so it has a budget of its own in the container's region: admitted with
// the same CAS loop and dead-process reclaim as device memory, released when the runtime
// frees or unlocks it, and dropped with the slot when a process exits.
//
// The HIP entry points keep only the reference's suspend gate.
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

#include <mutex>

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"
#include "vgpu/region.h"

using namespace vgpu;

namespace {

bool charge_host(size_t size) {
  ShimState& s = shim();
  if (s.region.charge_host(s.slot, size) == Charge::kOk) return true;
  VLOG_WARN("host memory OOM: request %zu bytes, pinned %lu of limit %lu", size, (unsigned long)s.region.host_usage(),
            (unsigned long)s.region.host_limit());
  return false;
}

// Records one more pin of `size` bytes at `p` (an allocation, or a lock of a user range):
// a re-lock of a pinned address keeps its own size, so the unlocks refund what was charged.
void record_host(void* p, uint64_t size) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  HostRec& h = s.host[reinterpret_cast<uintptr_t>(p)];
  h.pins.push_back(size);
  h.total += size;
}

bool accounting() {
  ShimState& s = shim();
  // ROCr initialised without passing the hsa_init hook: initialise on first use (hsa_hooks.cpp).
  if (__builtin_expect(s.phase.load(std::memory_order_acquire) == 0, 0)) shim_init_after_hsa();
  return s.phase.load(std::memory_order_acquire) == 2 && s.active && s.slot >= 0 && !s.exiting.load();
}

}  // namespace

namespace vgpu {

bool is_cpu_pool(hsa_amd_memory_pool_t pool) {
  const ShimState& s = shim();
  for (int i = 0; i < s.n_cpu_pools; i++)
    if (s.cpu_pools[i].handle == pool.handle) return true;
  return false;
}

hsa_status_t host_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  VGPU_REAL_HSA(hsa_amd_memory_pool_allocate);
  if (!size || !accounting() || !is_cpu_pool(pool)) return real_hsa_amd_memory_pool_allocate(pool, size, flags, ptr);
  gate_suspend();
  if (!charge_host(size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t st = real_hsa_amd_memory_pool_allocate(pool, size, flags, ptr);
  if (st != HSA_STATUS_SUCCESS || !ptr || !*ptr) {
    shim().region.uncharge_host(shim().slot, size);
    return st;
  }
  record_host(*ptr, size);
  return st;
}

bool take_host(void* p, HostRec* out) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  auto it = s.host.find(reinterpret_cast<uintptr_t>(p));
  if (it == s.host.end()) return false;
  *out = it->second;
  s.host.erase(it);
  return true;
}

void put_host(void* p, const HostRec& rec) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  HostRec& h = s.host[reinterpret_cast<uintptr_t>(p)];
  h.pins.insert(h.pins.begin(), rec.pins.begin(), rec.pins.end());
  h.total += rec.total;
}

uint64_t host_recorded_bytes() {
  ShimState& s = shim();
  uint64_t n = 0;
  for (const auto& kv : s.host) n += kv.second.total;
  return n;
}

}  // namespace vgpu

extern "C" {

// hsa_amd_memory_lock(_to_pool): pins a user range (hipHostRegister, or a direct ROCr
// caller). Charged before the real lock, refused past the budget.
hsa_status_t hsa_amd_memory_lock(void* host_ptr, size_t size, hsa_agent_t* agents, int num_agent, void** agent_ptr) {
  VGPU_REAL_HSA(hsa_amd_memory_lock);
  if (!real_hsa_amd_memory_lock) return HSA_STATUS_ERROR;
  if (!host_ptr || !size || !accounting()) return real_hsa_amd_memory_lock(host_ptr, size, agents, num_agent, agent_ptr);
  gate_suspend();
  if (!charge_host(size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t st = real_hsa_amd_memory_lock(host_ptr, size, agents, num_agent, agent_ptr);
  if (st != HSA_STATUS_SUCCESS) shim().region.uncharge_host(shim().slot, size);
  else record_host(host_ptr, size);
  return st;
}

hsa_status_t hsa_amd_memory_lock_to_pool(void* host_ptr, size_t size, hsa_agent_t* agents, int num_agent,
                                         hsa_amd_memory_pool_t pool, uint32_t flags, void** agent_ptr) {
  VGPU_REAL_HSA(hsa_amd_memory_lock_to_pool);
  if (!real_hsa_amd_memory_lock_to_pool) return HSA_STATUS_ERROR;
  if (!host_ptr || !size || !accounting())
    return real_hsa_amd_memory_lock_to_pool(host_ptr, size, agents, num_agent, pool, flags, agent_ptr);
  gate_suspend();
  if (!charge_host(size)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  hsa_status_t st = real_hsa_amd_memory_lock_to_pool(host_ptr, size, agents, num_agent, pool, flags, agent_ptr);
  if (st != HSA_STATUS_SUCCESS) shim().region.uncharge_host(shim().slot, size);
  else record_host(host_ptr, size);
  return st;
}

// One lock less: the latest pin's record is taken before the real unlock (a concurrent lock
// of the same address must not find it half-released), its own size refunded, and put back
// if the runtime refused. lock(p, 2G), lock(p, 1G), unlock, unlock refunds 1G then 2G.
hsa_status_t hsa_amd_memory_unlock(void* host_ptr) {
  VGPU_REAL_HSA(hsa_amd_memory_unlock);
  if (!real_hsa_amd_memory_unlock) return HSA_STATUS_ERROR;
  ShimState& s = shim();
  if (!host_ptr || s.phase.load(std::memory_order_acquire) != 2) return real_hsa_amd_memory_unlock(host_ptr);
  uint64_t pin = 0;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    auto it = s.host.find(reinterpret_cast<uintptr_t>(host_ptr));
    if (it != s.host.end() && !it->second.pins.empty()) {
      pin = it->second.pins.back();
      it->second.pins.pop_back();
      it->second.total -= pin;
      if (it->second.pins.empty()) s.host.erase(it);
    }
  }
  hsa_status_t st = real_hsa_amd_memory_unlock(host_ptr);
  if (!pin) return st;
  if (st != HSA_STATUS_SUCCESS) {
    record_host(host_ptr, pin);
    return st;
  }
  if (s.slot >= 0 && !s.exiting.load()) s.region.uncharge_host(s.slot, pin);
  return st;
}

}  // extern "C"

// ---------------------------------------------------------------- HIP entry points
// Suspend-gated pass-throughs: the memory they pin is charged in the ROCr calls above.

namespace {
using AllocFn3 = hipError_t (*)(void**, size_t, unsigned int);
using AllocFn2 = hipError_t (*)(void**, size_t);
using FreeFn = hipError_t (*)(void*);
using RegisterFn = hipError_t (*)(void*, size_t, unsigned int);
}  // namespace

#pragma GCC diagnostic push
#pragma GCC diagnostic ignored "-Wdeprecated-declarations"

extern "C" {

hipError_t hipHostMalloc(void** ptr, size_t size, unsigned int flags) {
  VGPU_REAL_AS(hipHostMalloc, AllocFn3, "libamdhip64", nullptr);
  if (!real_hipHostMalloc) return hipErrorNotSupported;
  gate_suspend();
  return real_hipHostMalloc(ptr, size, flags);
}

hipError_t hipHostAlloc(void** ptr, size_t size, unsigned int flags) {
  VGPU_REAL_AS(hipHostAlloc, AllocFn3, "libamdhip64", nullptr);
  if (!real_hipHostAlloc) return hipErrorNotSupported;
  gate_suspend();
  return real_hipHostAlloc(ptr, size, flags);
}

hipError_t hipMallocHost(void** ptr, size_t size) {
  VGPU_REAL_AS(hipMallocHost, AllocFn2, "libamdhip64", nullptr);
  if (!real_hipMallocHost) return hipErrorNotSupported;
  gate_suspend();
  return real_hipMallocHost(ptr, size);
}

hipError_t hipMemAllocHost(void** ptr, size_t size) {
  VGPU_REAL_AS(hipMemAllocHost, AllocFn2, "libamdhip64", nullptr);
  if (!real_hipMemAllocHost) return hipErrorNotSupported;
  gate_suspend();
  return real_hipMemAllocHost(ptr, size);
}

hipError_t hipHostFree(void* ptr) {
  VGPU_REAL_AS(hipHostFree, FreeFn, "libamdhip64", nullptr);
  if (!real_hipHostFree) return hipErrorNotSupported;
  gate_suspend();
  return real_hipHostFree(ptr);
}

hipError_t hipFreeHost(void* ptr) {
  VGPU_REAL_AS(hipFreeHost, FreeFn, "libamdhip64", nullptr);
  if (!real_hipFreeHost) return hipErrorNotSupported;
  gate_suspend();
  return real_hipFreeHost(ptr);
}

hipError_t hipHostRegister(void* host_ptr, size_t size, unsigned int flags) {
  VGPU_REAL_AS(hipHostRegister, RegisterFn, "libamdhip64", nullptr);
  if (!real_hipHostRegister) return hipErrorNotSupported;
  gate_suspend();
  return real_hipHostRegister(host_ptr, size, flags);
}

hipError_t hipHostUnregister(void* host_ptr) {
  VGPU_REAL_AS(hipHostUnregister, FreeFn, "libamdhip64", nullptr);
  if (!real_hipHostUnregister) return hipErrorNotSupported;
  gate_suspend();
  return real_hipHostUnregister(host_ptr);
}

}  // extern "C"

#pragma GCC diagnostic pop
