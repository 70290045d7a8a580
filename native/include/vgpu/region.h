// Per-container shared accounting region (mmap'd file shared by every process of a
// container, and optionally by a node monitor through a host path).
//
// Reference behaviour (libvgpu.so, src/multiprocess/multiprocess_memory_limit.c):
//   try_create_shrreg [645-741]  create/attach, init limits from env, verify consistency
//   lock_shrreg/fix_lock_shrreg  POSIX sem + "kick the dead owner" heuristic
//   init_proc_slot_withlock      <=1024 process slots, exit/atfork handlers
//   add/rm_gpu_device_memory_usage, get_gpu_memory_usage (sum over all slots)
//   rm_quitted_process           popen("ps a -o pid=") reclaim of dead slots
//   suspend_all/resume_all       SIGUSR2/SIGUSR1 broadcast
//
// MI355X-native redesign (not a layout copy):
//   * versioned header (magic + version + struct size) so a monitor can reject a
//     foreign layout instead of mis-reading it;
//   * robust process-shared pthread mutex (EOWNERDEAD -> consistent + reclaim)
//     instead of sem_timedwait + owner kick;
//   * a per-device aggregate `used` counter updated with a CAS admission loop, so the
//     OOM check is one atomic load and two concurrent allocators can never jointly
//     overshoot the quota (the reference sums 1024 slots without a lock);
//   * dead-process reclaim by kill(pid, 0) + /proc start-time check (PID reuse safe),
//     no subprocess;
//   * suspend/resume and the launch block are region state polled by the gates, so
//     the shim does not have to own SIGUSR1/SIGUSR2 in the user's process (opt-in
//     VGPU_SIGNAL_CONTROL keeps the signal protocol for parity);
//   * per-device CU mask + token bucket live in the region, so every process of a
//     container shares one compute budget.
#pragma once

#include <pthread.h>
#include <sys/types.h>

#include <atomic>
#include <cstddef>
#include <cstdint>

#include "vgpu/config.h"

namespace vgpu {

constexpr uint32_t kRegionMagic = 0x56475055u;  // "VGPU"
constexpr uint32_t kRegionVersion = 5;  // v5: pinned host memory accounting

enum ProcStatus : int32_t { kProcFree = 0, kProcRunning = 1, kProcSuspended = 2 };

// Memory categories tracked per process and device (reference: {context, module,
// data, offset, total} per device in each proc slot).
enum MemKind : int { kMemData = 0, kMemContext = 1, kMemModule = 2, kMemSpill = 3, kMemKinds = 4 };

struct alignas(64) DeviceUsage {
  std::atomic<uint64_t> total;            // sum of all kinds
  std::atomic<uint64_t> kind[kMemKinds];
  std::atomic<uint64_t> peak;
  // Bytes of this process's shared virtual memory in the device's VRAM (promoted spills, the
  // tenant's own prefetched ranges): HBM that ROCr's free-memory figure does not show
  // (profiles/r4b). Part of `kind[kMemData]`, not added to it. Published on the node board so
  // other containers see that HBM as taken.
  std::atomic<uint64_t> svm_vram;
};
// svm_vram sits in what was alignment padding in layout v5: the layout is unchanged.
static_assert(sizeof(DeviceUsage) == 64, "DeviceUsage layout changed");

struct alignas(64) ProcSlot {
  std::atomic<int32_t> pid;               // 0 = free slot
  std::atomic<int32_t> hostpid;           // PID in the host namespace (0 = unknown)
  std::atomic<int32_t> status;            // ProcStatus
  int32_t priority;
  uint64_t start_time;                    // /proc/<pid>/stat field 22, guards PID reuse
  std::atomic<uint64_t> launches;         // kernel launches through the gates
  std::atomic<uint64_t> throttle_ns;      // time spent blocked in the rate limiter
  std::atomic<uint64_t> suspend_ns;       // time spent blocked by suspend
  std::atomic<uint64_t> oom_events;
  uint64_t pidns;                         // inode of the PID namespace `pid` lives in (0 = unknown)
  DeviceUsage used[kMaxDevices];
  std::atomic<uint64_t> host_used;        // pinned host memory (hipHostMalloc / hipHostRegister)
  std::atomic<uint64_t> host_peak;
};
// pidns sits in what was alignment padding in layout v4: the layout is unchanged.
static_assert(offsetof(ProcSlot, used) == 64, "ProcSlot layout changed");

struct alignas(64) DeviceState {
  char uuid[64];
  uint64_t mem_limit;                     // bytes, 0 = unlimited
  uint64_t hbm_limit;                     // HBM-resident cap; beyond it allocations spill (0 = off)
  uint64_t phys_total;                    // physical HBM bytes reported by ROCr
  int32_t cu_limit_pct;                   // 0 / >=100 = unlimited
  int32_t cu_count;                       // physical CUs of the agent
  int32_t num_xcc;
  int32_t cu_mask_bits;                   // number of valid bits in cu_mask
  uint32_t cu_mask[kCuMaskWords];         // spatial mask applied to every queue
  std::atomic<uint64_t> used;             // aggregate bytes charged (all live slots)
  std::atomic<uint64_t> spilled;          // portion of `used` served from host memory
  std::atomic<uint64_t> monitor_used;     // sampled physical usage of the region's PIDs
  std::atomic<int64_t> credit_ns;         // temporal mode: GPU-time credit (ratelimit.h)
  std::atomic<uint64_t> charged_ns;       // GPU time charged to the container so far
  std::atomic<uint64_t> wall_ns;          // wall time the sampler has accounted
  std::atomic<int32_t> util_pm;           // smoothed utilisation, per mille
  std::atomic<int32_t> gate_open;         // temporal mode: launches may proceed
  int32_t num_se;                         // shader engines per XCC (mask layout)
  int32_t cu_range_begin;                 // logical CU range of the vGPU (-1 = from pct)
  int32_t cu_range_end;
  std::atomic<int32_t> cu_mode;           // effective CuMode of this device
  uint32_t gpu_id;                        // KFD gpu_id (stats_<gpu_id> in sysfs)
  uint32_t bdf;                           // PCI bus/device/function (HSA BDFID)
  uint32_t domain;                        // PCI domain
  uint32_t configured;                    // 1 once a GPU process filled the agent info
  std::atomic<int32_t> crowd;             // auto mode: other busy processes on the GPU (-1 = unknown)
  // Background class: CUs held by latency-class tenants on this GPU (their CU slices, from
  // the board); the container's queues keep off them (0 = none).
  uint32_t reserved_mask[kCuMaskWords];
  // Background class next to a better class (VGPU_PREEMPT_HOLD_MS / VGPU_PREEMPT_DEPTH):
  // launches held because a better class is busy, and the cap on the packets each process
  // of the container keeps in flight on this device (0 = none). Written by the sampler.
  std::atomic<int32_t> preempt;
  std::atomic<int32_t> depth_cap;
  // Exact GPU-time share of the limiter's grants, basis points (0 = cu_limit_pct): the
  // plugin's CU limit is a whole percent rounded up, so a split-16 vGPU's 6.25 % is 7 %.
  int32_t cu_share_bp;
  // Virtual device memory made visible node-wide (written by the container's sampler from the
  // node board): SVM bytes other containers hold in this GPU's VRAM, which ROCr's free-memory
  // figure does not show.
  std::atomic<uint64_t> node_svm_vram;
  // HBM pressure: this container was refused HBM within its share (hbm_want bytes, at
  // hbm_want_ns, CLOCK_MONOTONIC) - published on the board so co-tenants demote promoted
  // spills; and the bytes of its own promoted spills the container was asked to demote for
  // a co-tenant (its processes' migrators work it off).
  std::atomic<uint64_t> hbm_want;
  std::atomic<uint64_t> hbm_want_ns;
  std::atomic<uint64_t> demote_want;
};
// preempt / depth_cap / cu_share_bp and the fields after them sit in what was tail padding in
// layout v5: the layout is unchanged.
static_assert(sizeof(DeviceState) == 320, "DeviceState layout changed");

struct RegionHeader {
  uint32_t magic;
  uint32_t version;
  uint64_t region_size;                   // sizeof(Region) of the writer
  pthread_mutex_t mutex;                  // robust + process-shared
  std::atomic<int32_t> initialized;
  int32_t num_devices;
  std::atomic<int32_t> utilization_switch;  // 1 = temporal limiter on (reference init 1)
  std::atomic<int32_t> recent_kernel;       // < 0 blocks every launch (reference init 2)
  std::atomic<int32_t> priority;
  std::atomic<int32_t> proc_num;            // live slots
  std::atomic<int32_t> suspend_all;         // 1 = every gate blocks
  std::atomic<int32_t> watcher_pid;         // process that runs the utilisation watcher
  std::atomic<uint64_t> watcher_heartbeat;  // CLOCK_MONOTONIC ns of the last tick
  uint32_t flags;                           // RegionFlags
  std::atomic<uint32_t> other_refreshes;    // sampler reads of the other processes' occupancy
  std::atomic<uint64_t> generation;         // bumped on any limit change
  std::atomic<uint64_t> samples;            // sampler ticks (temporal mode)
  // Pinned host memory of the container (VGPU_HOST_MEMORY_LIMIT; reference: class (b)
  // cuMemAllocHost_v2 / cuMemHostAlloc / cuMemHostRegister_v2 OOM checks).
  uint64_t host_limit;                      // bytes, 0 = unlimited (tracked only)
  std::atomic<uint64_t> host_used;          // aggregate over live slots
  // Random tag written when the region is (re-)initialised: a process that finds another
  // epoch than the one it registered under knows its slot and charges were wiped (a tenant
  // rewriting its region) and registers and charges its live allocations again.
  uint64_t epoch;
};
// epoch sits in what was alignment padding before dev[] in layout v5: the layout is unchanged.
static_assert(offsetof(RegionHeader, epoch) + sizeof(uint64_t) <= 192, "RegionHeader grew into dev[]");

// Wait bound for the region lock on paths that must not hang behind a stopped holder.
constexpr int kLockTimeoutMs = 500;

enum RegionFlags : uint32_t { kFlagOversubscribe = 1u, kFlagActiveOomKiller = 2u };

struct Region {
  RegionHeader hdr;
  DeviceState dev[kMaxDevices];
  ProcSlot procs[kMaxProcs];
};

// Result of an admission check.
enum class Charge : int { kOk = 0, kOverLimit = 1 };

// A process's handle on an attached region.
class SharedRegion {
 public:
  SharedRegion() = default;
  ~SharedRegion();
  SharedRegion(const SharedRegion&) = delete;
  SharedRegion& operator=(const SharedRegion&) = delete;

  // Opens (creating if needed) and maps `path`. When the region is fresh, device
  // limits are initialised from `cfg`; when it exists, `cfg` is checked against the
  // stored limits ("Limit inconsistency detected" in the reference) and the stored
  // values win. Returns 0 or -errno.
  int attach(const char* path, const Config* cfg, bool create);
  void detach();
  bool attached() const { return r_ != nullptr; }
  Region* raw() { return r_; }
  const Region* raw() const { return r_; }
  const char* path() const { return path_; }

  // Robust lock. Returns false only if the mutex is unrecoverable.
  bool lock();
  // lock() that gives up after `timeout_ms` (false): for paths that must not hang behind
  // a lock holder that is alive but stopped (SIGSTOP, a debugger, a frozen cgroup). The
  // reference's lock_shrreg uses sem_timedwait for the same reason
  // (libvgpu.so lock_shrreg@0x4426a [multiprocess_memory_limit.c:516-540]).
  bool lock_for(int timeout_ms);
  void unlock();

  // Process slots.
  int register_process(pid_t pid, pid_t hostpid, int priority);  // slot index or -1
  void unregister_process(int slot);
  int find_slot(pid_t pid) const;
  int reclaim_dead();               // frees slots of exited processes, returns count

  // Accounting. charge() admits `bytes` on `dev` against the limit (CAS loop, with a
  // single reclaim-and-retry when over, as oom_check does in the reference).
  Charge charge(int slot, int dev, uint64_t bytes, MemKind kind);
  void uncharge(int slot, int dev, uint64_t bytes, MemKind kind);
  // Unconditional charge (used for memory the runtime already owns, e.g. a spill
  // fallback that must be recorded even past the limit).
  void force_charge(int slot, int dev, uint64_t bytes, MemKind kind);

  uint64_t usage(int dev) const;
  // The device's memory limit: the region's, lowered to this process's ceiling (0 = none).
  uint64_t limit(int dev) const;
  uint64_t hbm_limit(int dev) const;
  // Bytes of `dev` resident in HBM (charged minus spilled).
  uint64_t resident(int dev) const;
  uint64_t proc_usage(int slot, int dev) const;
  // Moves `bytes` of `dev` from spill to HBM-resident data (an SVM spill promoted into HBM)
  // if the container's resident bytes stay within `cap` (0 = no cap) - atomically with
  // respect to concurrent allocations of the container's other processes. False: not moved.
  bool promote_spill(int slot, int dev, uint64_t bytes, uint64_t cap);
  // The reverse (a promotion that failed after the move, or a demotion): data back to spill.
  void demote_to_spill(int slot, int dev, uint64_t bytes);
  // SVM bytes of `dev` in VRAM: this process's (published by it) and the container's sum.
  void set_svm_vram(int slot, int dev, uint64_t bytes);
  uint64_t svm_vram(int dev) const;

  // Pinned host memory (page-locked RAM is a node-wide resource the host-spill pool
  // shares): the same CAS admission with reclaim-and-retry as device memory.
  Charge charge_host(int slot, uint64_t bytes);
  void uncharge_host(int slot, uint64_t bytes);
  uint64_t host_usage() const;
  uint64_t host_limit() const;
  void set_host_limit(uint64_t bytes);

  // Process-local ceilings from the plugin's limits file (config.h load_ceiling): admission
  // never goes past them, whatever the shared region (which the tenant can write) says,
  // and set_limit / set_host_limit cannot raise a limit above them. 0 = no ceiling. Not
  // stored in the region.
  void set_ceiling(int dev, uint64_t mem_bytes);
  void set_host_ceiling(uint64_t bytes);
  // The HBM-resident share of an oversubscribed vGPU (VGPU_DEVICE_HBM_LIMIT_<i>): a tenant
  // writing 0 (no cap) into its region must not take the other tenants' HBM.
  void set_hbm_ceiling(int dev, uint64_t bytes);
  uint64_t ceiling(int dev) const { return dev >= 0 && dev < kMaxDevices ? ceil_mem_[dev] : 0; }
  uint64_t hbm_ceiling(int dev) const { return dev >= 0 && dev < kMaxDevices ? ceil_hbm_[dev] : 0; }
  // Re-initialises the mapped region in place when its header no longer holds a valid
  // layout (a tenant overwrote it); true if it did. Serialised with attach's file lock.
  bool reinit_if_invalid(const Config* cfg);
  // Inode of the region file (0 if unknown): checked against the plugin's record.
  uint64_t inode() const;
  // Sets the file's mtime to now (writes through the mapping need not): the plugin removes
  // region files untouched for an hour from its host directory.
  void touch();

  // External control API (reference: set_current_device_memory_limit,
  // set_current_device_sm_limit_scale, suspend_all, resume_all, priority,
  // recent_kernel).
  void set_limit(int dev, uint64_t bytes);
  // Changes the CU share of a device: the CU mask is recomputed here (every process of
  // the container re-applies it to its queues when it sees the generation change) and,
  // in auto mode, the enforcement mode follows the new share.
  void set_cu_limit(int dev, int pct);
  void suspend_all();
  void resume_all();
  void set_proc_status(int slot, int status);
  int num_devices() const;

 private:
  static void init_mutex(pthread_mutex_t* m);
  void init_fresh(const Config* cfg);
  void check_consistency(const Config* cfg);
  void clear_slot_locked(int slot);

  Region* r_ = nullptr;
  int fd_ = -1;
  char path_[512] = {0};
  uint64_t ceil_mem_[kMaxDevices] = {};
  uint64_t ceil_hbm_[kMaxDevices] = {};
  uint64_t ceil_host_ = 0;
};

// /proc/<pid>/stat start time (clock ticks since boot), 0 if unavailable.
uint64_t proc_start_time(pid_t pid);
// True if `pid` is alive and (when start_time != 0) is the same process.
bool proc_alive(pid_t pid, uint64_t start_time);
// Inode of the calling process's PID namespace (/proc/self/ns/pid), 0 if unreadable.
uint64_t self_pidns();
// The initial (host) PID namespace's inode (PROC_PID_INIT_INO).
constexpr uint64_t kInitPidNs = 0xEFFFFFFCull;

}  // namespace vgpu
