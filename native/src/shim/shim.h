// Process-wide state of the interception shim (libvgpu_hip.so).
//
// Reference init sequence: cuInit → preInit (load real driver
// table, nvmlInit, /overrideEnv, device map, shared region, visible devices) →
// real cuInit → postInit (allocmode, allocator, virtual PCI ids, host-PID discovery,
// utilisation watcher). Here the equivalent runs inside the hsa_init hook: every
// HIP program initialises ROCr exactly there, and the shim stays inert in processes
// that never touch the GPU (it is force-preloaded into every container process).
#pragma once

#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <atomic>
#include <cstdint>
#include <map>
#include <mutex>
#include <unordered_map>
#include <vector>

#include "vgpu/config.h"
#include "vgpu/cumask.h"
#include "vgpu/region.h"

namespace vgpu {

constexpr int kMaxAgentPools = 16;

struct AgentInfo {
  hsa_agent_t agent{0};
  hsa_agent_t cpu_agent{0};          // nearest CPU agent (host-spill pool owner)
  hsa_amd_memory_pool_t spill_pool{0};
  uint32_t gpu_id = 0;               // KFD gpu_id
  int cu_count = 0;
  int num_xcc = 1;
  int num_se = 1;                    // shader engines per XCC (mask layout)
  int max_waves_per_cu = 32;
  uint64_t phys_total = 0;
  std::atomic<bool> mask_active{false};      // spatial mask applied to its queues
  std::atomic<int> visible_cus{0};           // CU count reported to the runtime (0 = the real one)
  bool authorised = true;                    // listed in VGPU_ALLOWLIST (when one is configured)
  std::atomic<bool> temporal_active{false};  // GPU-time credit gates its launches
  CuMode mode = CuMode::kOff;                // effective enforcement mode
  CuMask mask;
  char uuid[64] = {0};                       // ROCr UUID ("GPU-...")
  // Plugin ceiling (limits file) for this agent: its CU share and slice; the region's may
  // only be narrower (0 = no ceiling).
  int ceil_pct = 0;
  int ceil_share_bp = 0;                     // exact GPU-time share of the file (basis points, 0 = none)
  CuMask ceil_mask;
  hsa_amd_memory_pool_t pools[kMaxAgentPools]{};  // GPU-local global pools (and regions) of this agent
  hsa_amd_memory_pool_t vram_pool{0};  // coarse-grained VRAM pool (host-PID probe allocations)
  int n_pools = 0;
};

struct AllocRec {
  uint64_t size;
  int dev;
  int kind;
};

// A spilled allocation backed by a KFD shared-virtual-memory range (spill.cpp): host RAM the
// GPU reaches in place until it is promoted into HBM, at the same address.
struct SvmRec {
  uint64_t size;      // bytes charged (the allocation's size)
  uint64_t mapped;    // bytes mapped (page-rounded)
  int dev;
  bool in_hbm;        // promoted: charged as HBM data, no longer as spill / host memory
  uint64_t seq;       // allocation order (oldest is promoted first)
  uint64_t retry_ns;  // a failed promotion is not retried before this time
};

// Pinned host memory of this process at one address (host_hooks.cpp): a CPU-pool allocation
// (one pin) or a user range locked once or more, each lock with its own size. Every pin is
// charged to the host budget by its own size; an unlock releases the latest pin (LIFO), a
// free all of them.
struct HostRec {
  uint64_t total = 0;           // bytes charged for the pins below
  std::vector<uint64_t> pins;   // each pin's size, oldest first
};

// A piece of a tenant's own SVM range (svm_hooks.cpp, hsa_amd_svm_attributes_set /
// hsa_amd_svm_prefetch_async): where the tenant asked it to live, and the device whose
// quota holds it (the prefetch location, else the preferred one; -1 = host memory).
struct TenantSvmSeg {
  uint64_t end;
  int pref;     // preferred location: device ordinal, -1 = host / none
  int loc;      // last prefetch target: device ordinal, -1 = host / none
  int charged;  // device charged for the bytes, -1 = none
};

struct ShimState {
  std::atomic<int> phase{0};         // 0 = not initialised, 1 = initialising, 2 = ready, 3 = inert
  bool active = false;               // accounting + gates enabled
  bool fail_closed = false;          // limits configured but no region: device memory refused
  SharedRegion region;
  int slot = -1;
  pid_t pid = 0;
  pid_t hostpid = 0;
  int n_agents = 0;
  AgentInfo agents[kMaxDevices];
  std::mutex alloc_mu;
  std::unordered_map<uintptr_t, AllocRec> allocs;   // device pointer → record
  std::unordered_map<uint64_t, AllocRec> vmem;      // vmem handle → record
  std::unordered_map<uintptr_t, AllocRec> managed;  // hipMallocManaged pointers charged at HIP level
  std::unordered_map<uintptr_t, AllocRec> ipc;      // IPC-attached pointers (owned by another process)
  std::unordered_map<uintptr_t, HostRec> host;      // pinned host memory (host_hooks.cpp)
  std::unordered_map<uintptr_t, AllocRec> vcharge;  // split duplicate vGPUs: the virtual slot charged (dev = slot)
  hsa_amd_memory_pool_t cpu_pools[kMaxAgentPools]{};  // global pools of the CPU agents (pinned host memory)
  int n_cpu_pools = 0;
  std::unordered_map<uintptr_t, int> queues;        // hsa_queue_t* → ordinal (under queue_mu)
  std::mutex queue_mu;                              // the queue map only: the crowded launch path reads
                                                    // it (wait_queue_depth) without meeting allocations
  std::unordered_map<uintptr_t, SvmRec> svm;        // SVM-backed spills (spill.cpp) → record
  std::mutex svm_mu;                                // serialises promotions with the frees of SVM spills
  int64_t svm_hbm[kMaxDevices] = {};                // promoted SVM bytes per device (under ctx_mu)
  int svm_kfd_vram = -1;                            // promoted SVM pages appear in KFD's vram_<gpu_id>: 1 / 0 / -1 unknown
  std::map<uintptr_t, TenantSvmSeg> tsvm;           // the tenant's own SVM ranges (svm_hooks.cpp), by start
  std::mutex tsvm_mu;
  int64_t tsvm_loc[kMaxDevices] = {};               // charged bytes prefetched onto a device (under ctx_mu)
  int64_t tsvm_pref[kMaxDevices] = {};              // charged bytes only preferred there (never in VRAM)
  std::atomic<bool> exiting{false};
  std::atomic<bool> watcher_started{false};
  std::atomic<uint64_t> seen_generation{0};         // region generation the queues reflect
  std::atomic<uint64_t> launches{0};                // published to the region by the maintenance thread
  std::atomic<bool> any_temporal{false};            // some agent is gated by the GPU-time limiter
  std::atomic<int64_t> ipc_bytes[kMaxDevices] = {};  // IPC-attached bytes per device
  std::mutex live_mu;                               // serialises live reconfiguration
  std::mutex ctx_mu;                                // serialises resync_context_charge
  std::atomic<void*> board_slot{nullptr};           // this process's mapping of the board slot (lease holder)
  Config resolved;                                  // per-agent config the region is (re-)initialised from
  uint64_t epoch = 0;                               // region epoch this process registered under
  bool has_ceiling = false;                         // a plugin limits file applies
};

ShimState& shim();

// Runs the one-time initialisation (after ROCr is up). Safe to call repeatedly.
void shim_init_after_hsa();
// Lightweight attach for processes that never initialise ROCr (e.g. amd-smi).
bool shim_attach_region_only();

// Per-hook call counters (diagnostics, VGPU_STATS=1 prints them at exit). Off by
// default: a disabled counter costs one predictable branch on a plain bool.
enum StatId : int {
  kStatAgentInfo, kStatPoolInfo, kStatAlloc, kStatFree, kStatQueueCreate, kStatCuMask,
  kStatLaunch, kStatGraphLaunch, kStatCopy, kStatSet, kStatCount
};
extern bool g_stats_on;
// Concurrency admission of this process's sampler (VGPU_STATS): turns taken, time held, time
// waited for them and the longest wait.
extern std::atomic<uint64_t> g_turns, g_turn_held_ns, g_turn_wait_ns, g_turn_wait_max_ns;
extern std::atomic<uint64_t> g_stats[kStatCount];
// Host waits (sync_hooks.cpp): blocking waits, of which polled, their time, poll wake-ups.
extern std::atomic<uint64_t> g_sync_waits, g_sync_polled, g_sync_wait_ns, g_sync_wakeups, g_sync_active,
    g_sync_active_ns;
#define VGPU_STAT(id)                                                                  \
  do {                                                                                 \
    if (__builtin_expect(::vgpu::g_stats_on, 0))                                       \
      ::vgpu::g_stats[::vgpu::id].fetch_add(1, std::memory_order_relaxed);             \
  } while (0)

// Ordinal of a GPU agent / pool, or -1.
int agent_ordinal(hsa_agent_t a);
int pool_ordinal(hsa_amd_memory_pool_t p);

// roctx ranges around blocking waits (trace.cpp; VGPU_TRACE=1).
void trace_push(const char* name);
void trace_pop();

// Suspend gate: blocks while the container is suspended (reference wait_status_self).
void gate_suspend_slow();
inline bool gate_needed() {
  ShimState& s = shim();
  if (__builtin_expect(!s.active || s.slot < 0, 1)) return false;
  Region* r = s.region.raw();
  return r->hdr.suspend_all.load(std::memory_order_relaxed) ||
         r->procs[s.slot].status.load(std::memory_order_relaxed) == kProcSuspended;
}
inline void gate_suspend() {
  if (__builtin_expect(gate_needed(), 0)) gate_suspend_slow();
}

// Kernel-launch gate: launch counter, live reconfiguration, suspend check, external
// launch block and the temporal GPU-time credit of device `dev` (dev < 0 = current HIP
// device).
void gate_launch(int dev);
// Packets of this process's queues on device `dev` the command processor has not taken yet.
uint64_t packets_queued(int dev);
// VGPU_HOOK_LAUNCH (gates.cpp): false turns the launch gates into pass-throughs.
extern bool g_launch_hooks_on;

// Waits (bounded) until this process's HSA queues on device `dev` hold at most `cap`
// AQL packets not yet consumed by the command processor (write - read index). Returns
// the nanoseconds waited.
uint64_t wait_queue_depth(int dev, int cap);

// Re-reads limits the controller changed in the region (generation bump): CU masks are
// re-applied to every tracked queue and the enforcement mode follows the new share.
void apply_live_config();
inline void check_live_config() {
  ShimState& s = shim();
  if (__builtin_expect(s.region.raw()->hdr.generation.load(std::memory_order_relaxed) !=
                           s.seen_generation.load(std::memory_order_relaxed),
                       0))
    apply_live_config();
}

// The container's task priority class as enforced: the region's (live, vgpuctl / monitor)
// raised to the plugin's floor (a tenant may write its region, not its limits file).
inline int effective_priority(const Region* r) {
  const int p = r->hdr.priority.load(std::memory_order_relaxed);
  const int floor = config().min_priority;
  return p < floor ? floor : p;
}

// Keeps the region within the plugin's ceilings (limits, HBM share, CU share and slice, host
// budget, priority floor): the tenant maps the region read-write, so whatever it wrote there is
// clamped back. Returns true if something was clamped. Called on attach and on every
// limit change (generation bump).
bool clamp_region_to_ceiling();

// A region whose epoch changed under this process (re-initialised, by a tenant rewriting
// it) no longer holds this process's slot or charges: re-registers and charges the live
// allocations the shim recorded again. Called by the maintenance thread every period.
void check_region_epoch();

// Per-process maintenance thread: host-PID discovery retries, continuous context
// accounting, and (for the process holding the container's sampler lease) the
// temporal-mode occupancy sampler, monitor-based usage and the active OOM killer.
void start_watcher_if_needed();

// Host PID of this process via the VRAM signature (kfd.h); 0 if still unknown.
pid_t resolve_hostpid(int lock_timeout_ms);

// Re-syncs this process's "context" charge on every device with KFD's view of its VRAM:
// context = vram_<gpu_id> − (tracked HBM allocations). Covers the
// runtime's internal allocations (queues, scratch / private segments, code objects)
// that never pass the pool hooks (reference: per-context and per-module charges,
// [context.c:49-86], [export_table.c:85-113]).
void resync_context_charge();

// Virtual device memory (spill.cpp). spill_allocate serves `size` bytes of device `dev`
// from host memory - a migratable SVM range when the driver has them (VGPU_SPILL_BACKING),
// else a pinned host-pool allocation - charged as spill and to the host budget, and records
// it. spill_release undoes it for a pointer the shim spilled (false: not a spill).
hsa_status_t spill_allocate(int dev, size_t size, void** ptr);
bool spill_release(void* ptr);
// Device memory of this process was freed: spills may fit into HBM now.
void notify_device_memory_freed();
// An SVM spill's GPU access list: hsa_amd_agents_allow_access on it (ROCr does not know the
// range) becomes SVM access attributes. Returns false if `ptr` is not an SVM spill.
bool svm_allow_access(const void* ptr, uint32_t n, const hsa_agent_t* agents, hsa_status_t* st);
// Bytes of SVM spills of `dev` promoted into HBM that KFD's VRAM counter does not show
// (resync_context_charge subtracts them from the tracked allocations).
int64_t svm_hbm_outside_kfd(int dev);
// HBM of `dev` that holds shared virtual memory - this container's promoted spills and
// prefetched ranges, and other containers' (node board) - when ROCr's free-memory figure does
// not show it (measured at the first migration; assumed until then, as on MI355X,
// profiles/r4b): taken off MEMORY_AVAIL wherever the shim decides by free HBM.
uint64_t hidden_vram(int dev);
// Stores this process's SVM bytes in each device's VRAM in its region slot (the sampler sums
// them for the node board). Called by the maintenance thread every period and after moves.
void publish_svm_vram();
// Physical HBM refused within the quota while co-tenants hold promoted spills on the GPU:
// asks them (node board) to demote spills and retries `attempt` until it succeeds or
// VGPU_DEMOTE_WAIT_MS passes. Returns the last status.
hsa_status_t reclaim_peer_hbm(int dev, size_t size, hsa_status_t (*attempt)(void*), void* ctx);
// Re-charges the SVM spills after the region was re-initialised (check_region_epoch).
void svm_recharge(int slot, uint64_t* host);
// Forgets the parent's SVM spills in a forked child (the ranges are not inherited).
void svm_forget();

// Pinned host memory (host_hooks.cpp), accounted where every path pins it: ROCr's CPU-pool
// allocations and memory locks. host_pool_allocate serves an allocation from a pool that is
// not a GPU's (charged to VGPU_HOST_MEMORY_LIMIT when it is a CPU pool).
// recorded). take_host removes the record of `p` (false: none) without uncharging it, for a
// caller that frees the memory next; put_host restores it when the free failed.
bool is_cpu_pool(hsa_amd_memory_pool_t pool);
hsa_status_t host_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr);
bool take_host(void* p, HostRec* out);
void put_host(void* p, const HostRec& rec);
// Sum of the recorded pinned bytes (re-charged after the region was re-initialised).
uint64_t host_recorded_bytes();

// The tenant's own SVM ranges (svm_hooks.cpp). A range placed on a GPU (preferred location
// or prefetch target) is admitted against that device's quota; moving it back to host
// memory or unmapping it releases the charge. svm_tenant_reconcile drops ranges the
// process unmapped (maintenance thread); svm_tenant_recharge re-charges them after the
// region was re-initialised; svm_tenant_forget clears them in a forked child.
void svm_tenant_reconcile();
void svm_tenant_recharge(int slot);
void svm_tenant_forget();
// Bytes of `dev` the tenant's SVM ranges hold that KFD's vram counter does not show.
int64_t svm_tenant_outside_kfd(int dev);
// Set while HIP allocates managed memory (hipMallocManaged charges it as a whole): the SVM
// calls the runtime makes for it are not charged again.
extern thread_local bool t_managed_alloc;

// The agent ordinal of HIP device `hipdev` (hipGetDevice / hipSetDevice numbering),
// matched by PCI address: HIP_VISIBLE_DEVICES inside the container may reorder or hide
// devices. Identity with one agent, or when the addresses are ambiguous (partitions).
int hip_device_agent(int hipdev);
// hip_device_agent of the calling thread's current HIP device (0 when unknown).
int current_hip_agent();

// Split duplicate vGPUs (vdev_hooks.cpp, VGPU_DUPLICATE_SPLIT): two vGPUs of one physical GPU
// are two HIP devices of the container, each with its own quota. vdev_split_active() is one
// relaxed load; vdev_to_phys maps a virtual ordinal to the physical one (negative ordinals -
// hipCpuDeviceId, hipInvalidDeviceId - and everything when split is off pass unchanged).
bool vdev_split_active();
int vdev_to_phys(int v);
// The region slot holding the quota of the virtual device the calling thread allocates on
// device (agent) `dev`, or -1 (no split, or no virtual device of that agent).
int vdev_charge_slot(int dev);

}  // namespace vgpu
