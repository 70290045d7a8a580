// ROCr (HSA) interposition: the single choke point for device memory, memory-info
// queries and queue creation on MI355X.
//
// Verified on box (profiles/shim_probe.md): libamdhip64 imports these entry points as
// `U sym@ROCR_1`; every hipMalloc / hipMallocAsync / library workspace reaches
// hsa_amd_memory_pool_allocate, hipMemGetInfo reads HSA_AMD_AGENT_INFO_MEMORY_AVAIL,
// and HIP's total memory comes from HSA_AMD_MEMORY_POOL_INFO_SIZE.
//
// Reference parity (libvgpu.so src/cuda/memory.c, src/allocator/allocator.c):
//   cuMemAlloc_v2 → suspend gate → oom_check → real alloc → add usage   (allocate)
//   cuMemFree_v2  → remove_chunk → rm usage                              (free)
//   cuMemGetInfo_v2 / cuDeviceTotalMem_v2 → limit-based answers          (info hooks)
//   CUDA_OVERSUBSCRIBE → managed memory                                  (host spill)
//   cuIpc* pass-through without double charge    (suspend-gated, charged to the exporter)
// MI355X-only: hsa_queue_create applies the vGPU's CU mask to every HW queue and
// hsa_amd_queue_cu_set_mask cannot widen it.
#include <time.h>
#include <unistd.h>

#include <dlfcn.h>

#include <algorithm>
#include <atomic>
#include <cstring>
#include <vector>

#include "real.h"
#include "shim.h"
#include "vgpu/kfd.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

using namespace vgpu;

namespace {

void record_alloc(uintptr_t key, uint64_t size, int dev, int kind) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  s.allocs[key] = AllocRec{size, dev, kind};
}

bool take_alloc(uintptr_t key, AllocRec* out) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.alloc_mu);
  auto it = s.allocs.find(key);
  if (it == s.allocs.end()) return false;
  *out = it->second;
  s.allocs.erase(it);
  return true;
}

// Placement of an allocation of a tenant with virtual device memory: true = host memory.
// First-come keeps HBM until the tenant's HBM share is used up. Large-first (default)
// sends large allocations (datasets, caches: bulk data touched a slice at a time) to host
// memory once they would eat into a reserve of the share, so the small, hot allocations
// that come later (weights, activations, workspaces) still find HBM; a large allocation
// also spills when the physical HBM (shared with other tenants) lacks size + reserve.
// Small allocations (below VGPU_SPILL_SMALL) may go a headroom past the share before they
// spill: a spilled buffer cannot be exported over IPC, and RCCL's transport buffers and the
// tensors a DataLoader worker shares are small ones allocated once the share may be full.
bool should_spill(int dev, size_t size) {
  ShimState& s = shim();
  const Config& cfg = config();
  const uint64_t hbm = s.region.hbm_limit(dev);
  if (!cfg.oversubscribe || !hbm) return false;
  // The caller has already charged `size` as data, so `resident` includes this request.
  const uint64_t resident = s.region.resident(dev);
  const bool large = cfg.spill_policy == SpillPolicy::kLargeFirst && size >= cfg.spill_large_bytes;
  if (!large) {
    if (resident <= hbm) return false;
    return size >= cfg.spill_small_bytes || resident > hbm + spill_small_headroom(cfg, hbm);
  }
  const uint64_t reserve = spill_reserve(cfg, hbm);
  if (resident + reserve > hbm) return true;
  VGPU_REAL_HSA(hsa_agent_get_info);
  uint64_t avail = 0;
  if (real_hsa_agent_get_info(s.agents[dev].agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MEMORY_AVAIL, &avail) !=
      HSA_STATUS_SUCCESS)
    return false;
  const uint64_t hidden = hidden_vram(dev);  // SVM pages in VRAM, node-wide: not in ROCr's figure
  avail = avail > hidden ? avail - hidden : 0;
  return avail < size + reserve;
}

// One real allocation attempt, retried by reclaim_peer_hbm while co-tenants demote.
struct PoolAttempt {
  hsa_amd_memory_pool_t pool;
  size_t size;
  uint32_t flags;
  void** ptr;
};
hsa_status_t pool_attempt(void* c) {
  VGPU_REAL_HSA(hsa_amd_memory_pool_allocate);
  const PoolAttempt* a = static_cast<const PoolAttempt*>(c);
  return real_hsa_amd_memory_pool_allocate(a->pool, a->size, a->flags, a->ptr);
}

// Limits are configured but the region could not be attached: GPU memory is refused.
inline bool refused(hsa_amd_memory_pool_t pool) {
  ShimState& s = shim();
  return __builtin_expect(s.fail_closed, 0) && pool_ordinal(pool) >= 0;
}

inline bool ready() {
  ShimState& s = shim();
  int ph = s.phase.load(std::memory_order_acquire);
  if (__builtin_expect(ph == 0, 0)) {
    // ROCr was initialised without going through our hsa_init hook (e.g. the shim
    // was loaded late); initialise on first use.
    shim_init_after_hsa();
    ph = s.phase.load(std::memory_order_acquire);
  }
  return ph == 2 && s.active && !s.exiting.load(std::memory_order_relaxed);
}

// The charge of an allocation on the calling thread's virtual device (split duplicate
// vGPUs, vdev_hooks.cpp): taken on construction, given back on destruction unless the
// allocation succeeded (commit records it for the free).
class VirtualCharge {
 public:
  VirtualCharge(int dev, size_t size) : size_(size) {
    ShimState& s = shim();
    slot_ = vdev_charge_slot(dev);
    if (slot_ >= 0 && s.region.charge(s.slot, slot_, size, kMemData) != Charge::kOk) {
      VLOG_WARN("virtual device (slot %d) OOM: request %zu bytes, usage %lu of limit %lu", slot_, size,
                (unsigned long)s.region.usage(slot_), (unsigned long)s.region.limit(slot_));
      failed_ = true;
    }
  }
  ~VirtualCharge() {
    if (slot_ >= 0 && !failed_ && !committed_) shim().region.uncharge(shim().slot, slot_, size_, kMemData);
  }
  bool ok() const { return !failed_; }
  void commit(void* p) const {
    if (slot_ < 0) return;
    committed_ = true;
    ShimState& s = shim();
    std::lock_guard<std::mutex> g(s.alloc_mu);
    s.vcharge[reinterpret_cast<uintptr_t>(p)] = AllocRec{size_, slot_, kMemData};
  }

 private:
  size_t size_;
  int slot_ = -1;
  bool failed_ = false;
  mutable bool committed_ = false;
};

}  // namespace

extern "C" {

hsa_status_t hsa_init() {
  VGPU_REAL_HSA(hsa_init);
  if (!real_hsa_init) return HSA_STATUS_ERROR;
  ShimState& s = shim();
  std::vector<int> before;
  bool first = s.phase.load() == 0;
  if (first) before = kfd_list_pids();
  hsa_status_t st = real_hsa_init();
  if (st == HSA_STATUS_SUCCESS && first) {
    if (!s.hostpid) {
      std::vector<int> after = kfd_list_pids();
      if (std::binary_search(after.begin(), after.end(), (int)getpid())) s.hostpid = getpid();
      else s.hostpid = kfd_diff_pid(before, after);
    }
    shim_init_after_hsa();
  }
  return st;
}

hsa_status_t hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  VGPU_REAL_HSA(hsa_amd_memory_pool_allocate);
  VGPU_STAT(kStatAlloc);
  if (!real_hsa_amd_memory_pool_allocate) return HSA_STATUS_ERROR;
  if (!ready() || size == 0) {
    if (size && refused(pool)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    return real_hsa_amd_memory_pool_allocate(pool, size, flags, ptr);
  }
  int dev = pool_ordinal(pool);
  VLOG_DEBUG("pool_allocate pool=%lx size=%zu flags=%u dev=%d", (unsigned long)pool.handle, size, flags, dev);
  if (dev < 0) return host_pool_allocate(pool, size, flags, ptr);  // pinned host memory (host_hooks.cpp)
  ShimState& s = shim();
  gate_suspend();
  if (__builtin_expect(!s.agents[dev].authorised, 0)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  if (s.region.charge(s.slot, dev, size, kMemData) != Charge::kOk) {
    VLOG_WARN("device %d OOM: request %zu bytes, usage %lu of limit %lu", dev, size,
              (unsigned long)s.region.usage(dev), (unsigned long)s.region.limit(dev));
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  // Split duplicate vGPUs: the calling thread's virtual device has its own quota too.
  const VirtualCharge vc(dev, size);
  if (!vc.ok()) {
    s.region.uncharge(s.slot, dev, size, kMemData);
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t st;
  // Virtual device memory: past the tenant's HBM-resident share the quota is served
  // from host memory (VGPU_DEVICE_HBM_LIMIT_<i>, emitted by the plugin when
  // --device-memory-scaling > 1), so one tenant cannot crowd the others out of HBM.
  if (should_spill(dev, size)) {
    st = spill_allocate(dev, size, ptr);  // charged as spill and recorded
    if (st == HSA_STATUS_SUCCESS) return vc.commit(*ptr), st;
    // No host memory for it: within the HBM share (an early, large-first spill) the
    // allocation may stay in HBM; past the share it is refused - the rest of the HBM
    // belongs to the other tenants of the GPU.
    if (s.region.resident(dev) > s.region.hbm_limit(dev)) {
      s.region.uncharge(s.slot, dev, size, kMemData);
      return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    }
  }
  st = real_hsa_amd_memory_pool_allocate(pool, size, flags, ptr);
  if (st == HSA_STATUS_ERROR_OUT_OF_RESOURCES) {
    // Within the quota but the GPU's HBM is full: co-tenants' promoted spills give it back.
    PoolAttempt at{pool, size, flags, ptr};
    st = reclaim_peer_hbm(dev, size, pool_attempt, &at);
  }
  if (st == HSA_STATUS_SUCCESS) {
    record_alloc(reinterpret_cast<uintptr_t>(*ptr), size, dev, kMemData);
    return vc.commit(*ptr), st;
  }
  if (st == HSA_STATUS_ERROR_OUT_OF_RESOURCES && config().oversubscribe) {
    // Under quota but the physical HBM is exhausted: virtual device memory.
    st = spill_allocate(dev, size, ptr);
    if (st == HSA_STATUS_SUCCESS) return vc.commit(*ptr), st;
  }
  s.region.uncharge(s.slot, dev, size, kMemData);
  return st;
}

// Split duplicate vGPUs: the allocation's charge on its virtual device goes with it.
static void release_virtual_charge(void* ptr) {
  ShimState& s = shim();
  AllocRec rec{0, -1, 0};
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    if (s.vcharge.empty()) return;
    auto it = s.vcharge.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == s.vcharge.end()) return;
    rec = it->second;
    s.vcharge.erase(it);
  }
  if (s.slot >= 0 && !s.exiting.load()) s.region.uncharge(s.slot, rec.dev, rec.size, kMemData);
}

// The one release path of both free entry points (ROCr accepts either for a pool or region
// allocation): an SVM spill is unmapped by the shim (ROCr never saw it); otherwise the
// record is taken before the runtime frees the memory - once freed, another thread may get
// the same address and record it - and the charges are dropped when the free succeeded
// (put back when it did not).
static hsa_status_t release_and_free(void* ptr, hsa_status_t (*real_free)(void*)) {
  ShimState& s = shim();
  if (!ptr || s.phase.load(std::memory_order_relaxed) != 2) return real_free(ptr);
  release_virtual_charge(ptr);
  if (spill_release(ptr)) return HSA_STATUS_SUCCESS;
  const uintptr_t key = reinterpret_cast<uintptr_t>(ptr);
  AllocRec rec{0, -1, 0};
  HostRec host;
  const bool dev_mem = take_alloc(key, &rec);
  const bool pinned = !dev_mem && take_host(ptr, &host);  // pinned host memory (host_hooks.cpp)
  hsa_status_t st = real_free(ptr);
  if (st != HSA_STATUS_SUCCESS) {
    if (dev_mem) record_alloc(key, rec.size, rec.dev, rec.kind);
    if (pinned) put_host(ptr, host);
    return st;
  }
  if (s.slot < 0 || s.exiting.load()) return st;
  if (dev_mem) {
    s.region.uncharge(s.slot, rec.dev, rec.size, (MemKind)rec.kind);
    if (rec.kind == kMemSpill) s.region.uncharge_host(s.slot, rec.size);  // a pinned spill
    else notify_device_memory_freed();
  }
  if (pinned) s.region.uncharge_host(s.slot, host.total);
  return st;
}

hsa_status_t hsa_amd_memory_pool_free(void* ptr) {
  VGPU_REAL_HSA(hsa_amd_memory_pool_free);
  VGPU_STAT(kStatFree);
  if (!real_hsa_amd_memory_pool_free) return HSA_STATUS_ERROR;
  return release_and_free(ptr, real_hsa_amd_memory_pool_free);
}

// The legacy region API reaches the same memory: ROCr's hsa_region_t and
// hsa_amd_memory_pool_t handles name the same memory-region objects (a GPU's coarse-grained
// VRAM region is its VRAM pool), so a region allocation is admitted like a pool allocation.
// ROCr serves it without passing through the exported pool entry point, so nothing is
// charged twice.
hsa_status_t hsa_memory_allocate(hsa_region_t region, size_t size, void** ptr) {
  VGPU_REAL_HSA(hsa_memory_allocate);
  if (!real_hsa_memory_allocate) return HSA_STATUS_ERROR;
  const hsa_amd_memory_pool_t pool{region.handle};
  if (!ready() || size == 0) {
    if (size && refused(pool)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    return real_hsa_memory_allocate(region, size, ptr);
  }
  int dev = pool_ordinal(pool);
  ShimState& s = shim();
  if (dev < 0) {
    // A CPU region: pinned host memory, charged to the host budget like a CPU-pool allocation.
    if (!is_cpu_pool(pool) || s.slot < 0) return real_hsa_memory_allocate(region, size, ptr);
    gate_suspend();
    if (s.region.charge_host(s.slot, size) != Charge::kOk) {
      VLOG_WARN("host memory OOM (region): request %zu bytes, pinned %lu of limit %lu", size,
                (unsigned long)s.region.host_usage(), (unsigned long)s.region.host_limit());
      return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    }
    hsa_status_t st = real_hsa_memory_allocate(region, size, ptr);
    if (st == HSA_STATUS_SUCCESS && ptr && *ptr) {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      HostRec& h = s.host[reinterpret_cast<uintptr_t>(*ptr)];
      h.pins.push_back(size);
      h.total += size;
    } else {
      s.region.uncharge_host(s.slot, size);
    }
    return st;
  }
  gate_suspend();
  if (__builtin_expect(!s.agents[dev].authorised, 0)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  if (s.region.charge(s.slot, dev, size, kMemData) != Charge::kOk) {
    VLOG_WARN("device %d OOM (region): request %zu bytes, usage %lu of limit %lu", dev, size,
              (unsigned long)s.region.usage(dev), (unsigned long)s.region.limit(dev));
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t st = real_hsa_memory_allocate(region, size, ptr);
  if (st == HSA_STATUS_SUCCESS && ptr && *ptr) record_alloc(reinterpret_cast<uintptr_t>(*ptr), size, dev, kMemData);
  else s.region.uncharge(s.slot, dev, size, kMemData);
  return st;
}

hsa_status_t hsa_memory_free(void* ptr) {
  VGPU_REAL_HSA(hsa_memory_free);
  if (!real_hsa_memory_free) return HSA_STATUS_ERROR;
  return release_and_free(ptr, real_hsa_memory_free);
}

// Peer access to a buffer (ROCclr grants it to the other GPUs of the process): an SVM spill
// is not a ROCr allocation, so its access list is set on the SVM range instead.
hsa_status_t hsa_amd_agents_allow_access(uint32_t num_agents, const hsa_agent_t* agents, const uint32_t* flags,
                                         const void* ptr) {
  VGPU_REAL_HSA(hsa_amd_agents_allow_access);
  if (!real_hsa_amd_agents_allow_access) return HSA_STATUS_ERROR;
  hsa_status_t st;
  if (ptr && shim().phase.load(std::memory_order_relaxed) == 2 && svm_allow_access(ptr, num_agents, agents, &st))
    return st;
  return real_hsa_amd_agents_allow_access(num_agents, agents, flags, ptr);
}

hsa_status_t hsa_amd_vmem_handle_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t type,
                                        uint64_t flags, hsa_amd_vmem_alloc_handle_t* handle) {
  VGPU_REAL_HSA(hsa_amd_vmem_handle_create);
  if (!real_hsa_amd_vmem_handle_create) return HSA_STATUS_ERROR;
  if (!ready() || size == 0) {
    if (size && refused(pool)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    return real_hsa_amd_vmem_handle_create(pool, size, type, flags, handle);
  }
  int dev = pool_ordinal(pool);
  if (dev < 0) return real_hsa_amd_vmem_handle_create(pool, size, type, flags, handle);
  ShimState& s = shim();
  gate_suspend();
  if (__builtin_expect(!s.agents[dev].authorised, 0)) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  if (s.region.charge(s.slot, dev, size, kMemData) != Charge::kOk) {
    VLOG_WARN("device %d OOM (vmem): request %zu bytes, usage %lu of limit %lu", dev, size,
              (unsigned long)s.region.usage(dev), (unsigned long)s.region.limit(dev));
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t st = real_hsa_amd_vmem_handle_create(pool, size, type, flags, handle);
  if (st != HSA_STATUS_SUCCESS) {
    s.region.uncharge(s.slot, dev, size, kMemData);
    return st;
  }
  std::lock_guard<std::mutex> g(s.alloc_mu);
  s.vmem[handle->handle] = AllocRec{size, dev, kMemData};
  return st;
}

hsa_status_t hsa_amd_vmem_handle_release(hsa_amd_vmem_alloc_handle_t handle) {
  VGPU_REAL_HSA(hsa_amd_vmem_handle_release);
  if (!real_hsa_amd_vmem_handle_release) return HSA_STATUS_ERROR;
  ShimState& s = shim();
  if (s.phase.load(std::memory_order_relaxed) == 2) {
    AllocRec rec{0, -1, 0};
    {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      auto it = s.vmem.find(handle.handle);
      if (it != s.vmem.end()) {
        rec = it->second;
        s.vmem.erase(it);
      }
    }
    if (rec.dev >= 0 && s.slot >= 0 && !s.exiting.load()) {
      s.region.uncharge(s.slot, rec.dev, rec.size, kMemData);
      notify_device_memory_freed();
    }
  }
  return real_hsa_amd_vmem_handle_release(handle);
}

hsa_status_t hsa_amd_memory_pool_get_info(hsa_amd_memory_pool_t pool, hsa_amd_memory_pool_info_t attr, void* value) {
  VGPU_REAL_HSA(hsa_amd_memory_pool_get_info);
  VGPU_STAT(kStatPoolInfo);
  if (!real_hsa_amd_memory_pool_get_info) return HSA_STATUS_ERROR;
  hsa_status_t st = real_hsa_amd_memory_pool_get_info(pool, attr, value);
  if (st != HSA_STATUS_SUCCESS || attr != HSA_AMD_MEMORY_POOL_INFO_SIZE || !value) return st;
  if (!ready()) return st;
  int dev = pool_ordinal(pool);
  if (dev < 0) return st;
  uint64_t lim = shim().region.limit(dev);
  if (!lim) return st;
  size_t* v = static_cast<size_t*>(value);
  // Virtual device memory: with oversubscription the quota may exceed the HBM and
  // is reported as is (reference: total = limit in cuDeviceTotalMem/cuMemGetInfo).
  if (config().oversubscribe || lim < *v) *v = (size_t)lim;
  return st;
}

hsa_status_t hsa_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  VGPU_REAL_HSA(hsa_agent_get_info);
  VGPU_STAT(kStatAgentInfo);
  if (!real_hsa_agent_get_info) return HSA_STATUS_ERROR;
  hsa_status_t st = real_hsa_agent_get_info(agent, attr, value);
  if (((int)attr == HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT ||
       (int)attr == HSA_AMD_AGENT_INFO_COOPERATIVE_COMPUTE_UNIT_COUNT) && st == HSA_STATUS_SUCCESS) {
    // Reference: cuDeviceGetAttribute virtualisation [device.c:130-134]. Here the CU
    // count follows the spatial slice (AgentInfo::visible_cus), read once by CLR at init
    // (its maxComputeUnits / hipDeviceProp multiProcessorCount come from the cooperative
    // count, the total CU count from the other attribute).
    const bool r = ready();
    int dev = r ? agent_ordinal(agent) : -1;
    int n = dev >= 0 ? shim().agents[dev].visible_cus.load(std::memory_order_relaxed) : 0;
    VLOG_DEBUG("agent_info CU count (attr %#x): dev=%d real=%u visible=%d", (unsigned)attr, dev,
               *static_cast<uint32_t*>(value), n);
    if (n > 0 && (uint32_t)n < *static_cast<uint32_t*>(value)) *static_cast<uint32_t*>(value) = (uint32_t)n;
    return st;
  }
  if (__builtin_expect((int)attr != HSA_AMD_AGENT_INFO_MEMORY_AVAIL, 1) || st != HSA_STATUS_SUCCESS) return st;
  if (!ready()) return st;
  int dev = agent_ordinal(agent);
  if (dev < 0) return st;
  ShimState& s = shim();
  uint64_t lim = s.region.limit(dev);
  if (!lim) return st;
  uint64_t used = s.region.usage(dev);
  uint64_t avail = lim > used ? lim - used : 0;
  uint64_t* v = static_cast<uint64_t*>(value);
  if (!config().oversubscribe) {
    // Other tenants may hold HBM - SVM pages in VRAM too, which ROCr's figure leaves out
    // (this container's and, from the node board, the other containers').
    const uint64_t hidden = hidden_vram(dev);
    const uint64_t phys = *v > hidden ? *v - hidden : 0;
    if (phys < avail) avail = phys;
  }
  *v = avail;
  return st;
}

hsa_status_t hsa_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                              void (*callback)(hsa_status_t, hsa_queue_t*, void*), void* data,
                              uint32_t private_segment_size, uint32_t group_segment_size, hsa_queue_t** queue) {
  VGPU_REAL_HSA(hsa_queue_create);
  VGPU_STAT(kStatQueueCreate);
  if (!real_hsa_queue_create) return HSA_STATUS_ERROR;
  hsa_status_t st =
      real_hsa_queue_create(agent, size, type, callback, data, private_segment_size, group_segment_size, queue);
  if (st != HSA_STATUS_SUCCESS || !queue || !*queue || !ready()) return st;
  int dev = agent_ordinal(agent);
  if (dev < 0) return st;
  ShimState& s = shim();
  AgentInfo& a = s.agents[dev];
  {
    std::lock_guard<std::mutex> g(s.queue_mu);
    s.queues[reinterpret_cast<uintptr_t>(*queue)] = dev;
  }
  if (a.mask_active.load()) {
    VGPU_REAL_HSA(hsa_amd_queue_cu_set_mask);
    uint32_t nbits = (uint32_t)((a.cu_count + 31) / 32 * 32);
    hsa_status_t ms = real_hsa_amd_queue_cu_set_mask(*queue, nbits, a.mask.words);
    if (ms != HSA_STATUS_SUCCESS && (int)ms != (int)HSA_STATUS_CU_MASK_REDUCED)
      VLOG_ERROR("device %d: cannot apply CU mask to queue %p (status %d)", dev, (void*)*queue, (int)ms);
    else
      VLOG_DEBUG("device %d: queue %p confined to %d CUs", dev, (void*)*queue, a.mask.count());
  }
  // Task priority (reference CUDA_TASK_PRIORITY, only stored there) becomes the hardware
  // queue priority: 0 = high (e.g. latency-critical inference next to batch jobs),
  // 1 = normal (default), >= 2 = low. Read from the region so an operator can change it.
  int prio = effective_priority(s.region.raw());
  if (prio != 1) {
    VGPU_REAL_HSA(hsa_amd_queue_set_priority);
    hsa_amd_queue_priority_t qp = prio <= 0 ? HSA_AMD_QUEUE_PRIORITY_HIGH : HSA_AMD_QUEUE_PRIORITY_LOW;
    if (real_hsa_amd_queue_set_priority && real_hsa_amd_queue_set_priority(*queue, qp) != HSA_STATUS_SUCCESS)
      VLOG_WARN("device %d: cannot set queue priority %d", dev, (int)qp);
    else
      VLOG_INFO("device %d: queue %p priority %s", dev, (void*)*queue, prio <= 0 ? "high" : "low");
  }
  // Queue creation is where ROCr allocates the process's ring buffers, scratch and
  // trap handlers: account them right away (the maintenance thread keeps it in sync).
  resync_context_charge();
  return st;
}

hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* queue, uint32_t num_cu_mask_count, const uint32_t* cu_mask) {
  VGPU_REAL_HSA(hsa_amd_queue_cu_set_mask);
  VGPU_STAT(kStatCuMask);
  if (!real_hsa_amd_queue_cu_set_mask) return HSA_STATUS_ERROR;
  if (!ready()) return real_hsa_amd_queue_cu_set_mask(queue, num_cu_mask_count, cu_mask);
  ShimState& s = shim();
  int dev = -1;
  {
    std::lock_guard<std::mutex> g(s.queue_mu);
    auto it = s.queues.find(reinterpret_cast<uintptr_t>(queue));
    if (it != s.queues.end()) dev = it->second;
  }
  if (dev < 0 || !s.agents[dev].mask_active.load())
    return real_hsa_amd_queue_cu_set_mask(queue, num_cu_mask_count, cu_mask);
  AgentInfo& a = s.agents[dev];
  // A user mask (hipExtStreamCreateWithCUMask, ROC_GLOBAL_CU_MASK) may only narrow
  // the vGPU's partition, never widen it; count 0 means "all CUs" → the vGPU mask.
  CuMask user;
  user.nbits = a.cu_count;
  if (num_cu_mask_count == 0 || !cu_mask) {
    user = a.mask;
  } else {
    for (uint32_t i = 0; i < num_cu_mask_count && i < (uint32_t)kMaxCUs; i++)
      if ((cu_mask[i / 32] >> (i % 32)) & 1u) user.set((int)i);
  }
  CuMask eff = cu_mask_intersect(user, a.mask, a.num_xcc);
  uint32_t nbits = (uint32_t)((a.cu_count + 31) / 32 * 32);
  return real_hsa_amd_queue_cu_set_mask(queue, nbits, eff.words);
}

}  // extern "C"

namespace vgpu {

namespace {

// Packets of this process's queues on `dev` the CP has not consumed yet. The queue map's
// own lock (not the allocation lock: this runs on every gated launch of a crowded GPU)
// keeps hsa_queue_destroy (which erases under it first) from freeing a queue while
// its indices are read.
uint64_t queued_packets(int dev) {
  VGPU_REAL_HSA(hsa_queue_load_write_index_relaxed);
  VGPU_REAL_HSA(hsa_queue_load_read_index_relaxed);
  if (!real_hsa_queue_load_write_index_relaxed || !real_hsa_queue_load_read_index_relaxed) return 0;
  ShimState& s = shim();
  uint64_t n = 0;
  std::lock_guard<std::mutex> g(s.queue_mu);
  for (const auto& q : s.queues) {
    if (q.second != dev) continue;
    const hsa_queue_t* h = reinterpret_cast<const hsa_queue_t*>(q.first);
    const uint64_t w = real_hsa_queue_load_write_index_relaxed(h), rd = real_hsa_queue_load_read_index_relaxed(h);
    if (w > rd) n += w - rd;
  }
  return n;
}

}  // namespace

uint64_t packets_queued(int dev) { return queued_packets(dev); }

uint64_t wait_queue_depth(int dev, int cap) {
  // Bounded: a queue can also hold packets that wait on something only this thread would
  // launch later (a barrier on another stream's event), which must never deadlock.
  constexpr uint64_t kMaxWaitNs = 20'000'000ull;
  if (queued_packets(dev) <= (uint64_t)cap) return 0;
  const uint64_t t0 = now_ns();
  trace_push("vgpu:depth");
  // Sleeps grow with the time waited (1/8 of it, 20 us to 500 us), as the host waits do
  // (sync_hooks.cpp): a long drain costs a few dozen wake-ups, not a core.
  for (uint64_t el = 0; queued_packets(dev) > (uint64_t)cap && el < kMaxWaitNs; el = now_ns() - t0) {
    struct timespec ts = {0, (long)std::min<uint64_t>(std::max<uint64_t>(el / 8, 20'000), 500'000)};
    nanosleep(&ts, nullptr);
  }
  trace_pop();
  return now_ns() - t0;
}

}  // namespace vgpu

extern "C" {

hsa_status_t hsa_queue_destroy(hsa_queue_t* queue) {
  VGPU_REAL_HSA(hsa_queue_destroy);
  if (!real_hsa_queue_destroy) return HSA_STATUS_ERROR;
  ShimState& s = shim();
  if (s.phase.load(std::memory_order_relaxed) == 2) {
    std::lock_guard<std::mutex> g(s.queue_mu);
    s.queues.erase(reinterpret_cast<uintptr_t>(queue));
  }
  return real_hsa_queue_destroy(queue);
}

// IPC (reference: cuIpcOpenMemHandle/CloseMemHandle are suspend-gated pass-throughs,
// [memory.c:374-388]). The exporting process already holds the charge for the buffer
// and KFD does not count the import in the importer's VRAM, so the importer is never
// charged; the mapping is recorded for diagnostics (VGPU_LOG_LEVEL=4, ipc_bytes).
hsa_status_t hsa_amd_ipc_memory_attach(const hsa_amd_ipc_memory_t* handle, size_t len, uint32_t num_agents,
                                       const hsa_agent_t* mapping_agents, void** mapped_ptr) {
  VGPU_REAL_HSA(hsa_amd_ipc_memory_attach);
  if (!real_hsa_amd_ipc_memory_attach) return HSA_STATUS_ERROR;
  gate_suspend();
  hsa_status_t st = real_hsa_amd_ipc_memory_attach(handle, len, num_agents, mapping_agents, mapped_ptr);
  if (st != HSA_STATUS_SUCCESS || !mapped_ptr || !*mapped_ptr || !ready()) return st;
  ShimState& s = shim();
  int dev = num_agents && mapping_agents ? agent_ordinal(mapping_agents[0]) : 0;
  if (dev < 0) dev = 0;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    s.ipc[reinterpret_cast<uintptr_t>(*mapped_ptr)] = AllocRec{len, dev, kMemData};
  }
  s.ipc_bytes[dev].fetch_add((int64_t)len);
  VLOG_DEBUG("ipc attach %zu bytes at %p on device %d (charged to the exporter)", len, *mapped_ptr, dev);
  return st;
}

hsa_status_t hsa_amd_ipc_memory_detach(void* mapped_ptr) {
  VGPU_REAL_HSA(hsa_amd_ipc_memory_detach);
  if (!real_hsa_amd_ipc_memory_detach) return HSA_STATUS_ERROR;
  ShimState& s = shim();
  if (mapped_ptr && s.phase.load(std::memory_order_relaxed) == 2) {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    auto it = s.ipc.find(reinterpret_cast<uintptr_t>(mapped_ptr));
    if (it != s.ipc.end()) {
      s.ipc_bytes[it->second.dev].fetch_sub((int64_t)it->second.size);
      s.ipc.erase(it);
    }
  }
  return real_hsa_amd_ipc_memory_detach(mapped_ptr);
}

}  // extern "C"

namespace vgpu {

// Every ROCr entry point the shim defines (libvgpu_hip.map.in, ROCR_1). Lookups of these
// names on a libhsa-runtime64 handle are routed here (dlsym_hook.cpp).
const char* const kHsaHooked[] = {
    "hsa_init", "hsa_amd_memory_pool_allocate", "hsa_amd_memory_pool_free", "hsa_amd_memory_pool_get_info",
    "hsa_amd_vmem_handle_create", "hsa_amd_vmem_handle_release", "hsa_agent_get_info", "hsa_queue_create",
    "hsa_queue_destroy", "hsa_amd_queue_cu_set_mask", "hsa_amd_ipc_memory_attach", "hsa_amd_ipc_memory_detach",
    "hsa_memory_allocate", "hsa_memory_free", "hsa_amd_agents_allow_access",
    "hsa_amd_svm_attributes_set", "hsa_amd_svm_prefetch_async",  // svm_hooks.cpp
    "hsa_amd_memory_lock", "hsa_amd_memory_lock_to_pool", "hsa_amd_memory_unlock",  // host_hooks.cpp
    "hsa_signal_wait_scacquire",                                                       // sync_hooks.cpp
};
constexpr int kNumHsaHooked = sizeof(kHsaHooked) / sizeof(kHsaHooked[0]);

void* hsa_hook_for_name(const char* name) {
  // The shim's own definitions, by symbol version from its own handle (and checked to lie
  // in the shim: a lookup on the shim's handle also searches its dependencies).
  static std::atomic<void*> self[kNumHsaHooked];
  static std::once_flag once;
  std::call_once(once, [] {
    Dl_info me;
    if (!dladdr(reinterpret_cast<void*>(&hsa_hook_for_name), &me) || !me.dli_fname) return;
    void* h = dlopen(me.dli_fname, RTLD_NOLOAD | RTLD_LAZY);
    if (!h) return;
    for (int i = 0; i < kNumHsaHooked; i++) {
      void* p = real_dlvsym(h, kHsaHooked[i], "ROCR_1");
      Dl_info di;
      if (p && dladdr(p, &di) && di.dli_fbase == me.dli_fbase) self[i].store(p, std::memory_order_relaxed);
    }
    dlclose(h);
  });
  for (int i = 0; i < kNumHsaHooked; i++)
    if (strcmp(kHsaHooked[i], name) == 0) return self[i].load(std::memory_order_relaxed);
  return nullptr;
}

}  // namespace vgpu
