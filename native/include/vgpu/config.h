// Container-side configuration of the vGPU shim, parsed once from the environment.
//
// This is the consumer half of the plugin→shim ABI. The reference
// reads CUDA_DEVICE_MEMORY_LIMIT[_i], CUDA_DEVICE_SM_LIMIT, NVIDIA_DEVICE_MAP,
// CUDA_DEVICE_MEMORY_SHARED_CACHE, CUDA_OVERSUBSCRIBE, CUDA_TASK_PRIORITY,
// GPU_CORE_UTILIZATION_POLICY, ACTIVE_OOM_KILLER and MEMORY_OVERRIDE
// (libvgpu.so:get_limit_from_env [multiprocess_memory_limit.c:101-111],
// postInit@0x16ded, set_env_utilization_switch@0x569dc). The MI355X names are the
// VGPU_* equivalents, plus the CU range the plugin assigns for spatial partitioning.
#pragma once

#include <cstdint>
#include <string>

namespace vgpu {

constexpr int kMaxDevices = 16;     // same hard cap as the reference (virtual_map[16])
constexpr int kMaxProcs = 1024;     // process slots per region (reference: cmp 0x3ff)
constexpr int kMaxCUs = 256;        // MI355X: 8 XCDs x 32 CUs
constexpr int kCuMaskWords = kMaxCUs / 32;

// How the CU share (VGPU_DEVICE_CU_LIMIT) is enforced.
enum class CuMode : int {
  kOff = 0,       // no compute limit
  kSpatial = 1,   // per-queue CU mask (hsa_amd_queue_cu_set_mask): default on MI355X
  kTemporal = 2,  // GPU-time credit checked at kernel launch (ratelimit.h)
  kBoth = 3,
  kAuto = 4,      // spatial for shares >= 50 %; below, spatial unless the GPU is crowded (effective_cu_mode)
};

// Spatial masks serve at most two co-resident tenants well: beyond that the tenants'
// dispatches contend in the shared front end (profiles/r1z), so smaller shares are
// enforced in time instead (profiles/r2*/scaling.md).
constexpr int kAutoSpatialMinPct = 50;
// Auto mode below kAutoSpatialMinPct: CU masks while at most this many other processes
// keep the GPU busy (masked tenants only stall each other in the dispatchers from about
// four on), the GPU-time limiter beyond.
constexpr int kAutoSpatialMaxCrowd = 1;
// The mode a device actually uses for share `pct` under configured mode `m`.
// `crowd`: other busy processes on the GPU (-1 = unknown, treated as crowded).
CuMode effective_cu_mode(CuMode m, int pct, int crowd = -1);
// Auto mode with the task priority class (VGPU_TASK_PRIORITY, vgpu/board.h): the latency
// class (<= 0) is never duty-cycled - its share stays a CU mask however crowded the GPU;
// the background class (>= 2) runs on the GPU-time gate whenever another process keeps
// the GPU busy (it yields to busier higher-priority tenants there), even without a limit.
CuMode effective_cu_mode_prio(CuMode m, int pct, int crowd, int priority);

// Where oversubscribed allocations live (VGPU_SPILL_POLICY).
enum class SpillPolicy : int {
  kFirstCome = 0,   // HBM until the tenant's HBM share is used up, then host memory
  kLargeFirst = 1,  // large allocations spill first; a reserve of the share stays for small ones
};

// What backs a spilled allocation (VGPU_SPILL_BACKING).
enum class SpillBacking : int {
  kAuto = 0,    // large allocations (>= VGPU_SPILL_LARGE): a migratable SVM range when the driver
                // supports it; smaller ones: pinned host memory, else SVM
  kSvm = 1,     // (default) KFD shared virtual memory: pageable host RAM mapped into the GPU in
                // place, migrated into HBM (same address) when the tenant's HBM share frees up;
                // pinned host memory where the driver has no SVM
  kPinned = 2,  // a pinned host-pool allocation (never moves)
};

// How the temporal limiter charges a container that shares the GPU (VGPU_CHARGE_MODEL).
enum class ChargeModel : int {
  kShare = 0,     // wall time x its share of the resident waves (processor sharing)
  kProgress = 1,  // at least wall time x its waves relative to its own recent peak: a
                  // tenant that co-runs without losing occupancy pays what it would alone
};

// Host waits of a HIP process (VGPU_SYNC_WAIT, native/src/shim/sync_hooks.cpp).
enum class SyncWait : int {
  kAuto = 0,    // poll with short sleeps while the GPU is crowded, else the runtime's own wait
  kPoll = 1,    // always poll
  kNative = 2,  // never (the runtime's wait, which spins a CPU)
};

// GPU_CORE_UTILIZATION_POLICY analogue.
enum class CuPolicy : int { kDefault = 0, kForce = 1, kDisable = 2 };

struct DeviceConfig {
  uint64_t mem_limit = 0;      // bytes, 0 = unlimited
  uint64_t hbm_limit = 0;      // HBM-resident cap (oversubscription), 0 = mem_limit
  int cu_limit_pct = 0;        // 0 or >= 100 = unlimited
  int cu_share_bp = 0;         // VGPU_DEVICE_CU_SHARE_<i>: exact GPU-time share in basis points for the
                               // limiter's grants (0 = cu_limit_pct); the plugin sends it with --ledger
  int cu_range_begin = -1;     // explicit logical CU range [begin, end) or -1 = derive
  int cu_range_end = -1;
  char uuid[64] = {0};         // physical UUID from VGPU_DEVICE_MAP (may be empty)
  bool unmapped = false;       // agent absent from a non-empty VGPU_DEVICE_MAP: not this container's
};

struct Config {
  bool disabled = false;                 // VGPU_DISABLE=1: shim is fully inert
  int num_devices = 0;                   // devices that carry an explicit config
  DeviceConfig dev[kMaxDevices];
  std::string shared_cache = "/tmp/vgpushr.cache";
  bool oversubscribe = false;            // VGPU_OVERSUBSCRIBE
  SpillPolicy spill_policy = SpillPolicy::kLargeFirst;  // VGPU_SPILL_POLICY
  uint64_t spill_large_bytes = 256ull << 20;  // VGPU_SPILL_LARGE: "large" allocation threshold
  uint64_t spill_reserve_bytes = 0;      // VGPU_SPILL_RESERVE: HBM kept for small ones (0 = auto)
  uint64_t spill_small_bytes = 64ull << 20;  // VGPU_SPILL_SMALL: below this an allocation may use the headroom
  int64_t spill_small_headroom = -1;     // VGPU_SPILL_SMALL_HEADROOM: HBM above the share for them (-1 = auto)
  SpillBacking spill_backing = SpillBacking::kSvm;  // VGPU_SPILL_BACKING: svm | auto | pinned
  bool spill_promote = true;             // VGPU_SPILL_PROMOTE: move SVM spills into HBM once they fit
  int demote_wait_ms = 2000;             // VGPU_DEMOTE_WAIT_MS: HBM refused within the quota - wait this
                                         // long for co-tenants to demote promoted spills (0 = never)
  int priority = 1;                      // VGPU_TASK_PRIORITY
  CuMode cu_mode = CuMode::kAuto;        // VGPU_CU_MODE
  CuPolicy cu_policy = CuPolicy::kDefault;
  bool active_oom_killer = true;         // VGPU_ACTIVE_OOM_KILLER (reference default: on)
  SyncWait sync_wait = SyncWait::kAuto;  // VGPU_SYNC_WAIT: auto | poll | native
  bool memory_override = false;          // VGPU_MEMORY_OVERRIDE
  bool signal_control = false;           // VGPU_SIGNAL_CONTROL: also honour SIGUSR1/2
  bool hook_smi = true;                  // VGPU_HOOK_SMI: virtualise amd-smi/rocm-smi
  bool virtual_cu_count = true;          // VGPU_VIRTUAL_CU_COUNT: report the spatial slice's CUs
  int auto_min_slice_cus = 40;           // VGPU_AUTO_MIN_SLICE_CUS: in auto mode a share whose CU slice is
                                         // thinner (at most 4 CUs per XCD: split >= 7 of 256 CUs) is time-sliced
                                         // only - never a mask - and the runtime sees every CU (0 = any width)
  int util_period_ms = 120;              // monitor / OOM-killer / accounting period (reference: 120 ms)
  int util_sample_us = 1000;             // temporal-mode occupancy sampling interval
  int sample_read_budget = 32;           // node-wide occupancy reads per interval (ratelimit.h)
  int limiter_window_ms = 40;            // temporal-mode credit window (ratelimit.h)
  int limiter_solo_window_ms = 160;      // VGPU_LIMITER_SOLO_WINDOW_MS: the window while no other process
                                         // keeps the GPU busy (longer on/off periods, fewer warm-ups; 0 = off)
  ChargeModel charge_model = ChargeModel::kShare;  // VGPU_CHARGE_MODEL: share | progress
  std::string board_dir;                 // VGPU_BOARD_DIR: node-wide board (vgpu/board.h), "" = none
  std::string board_slot;                // VGPU_BOARD_SLOT: this container's slot file in it
  int gpu_concurrency = 0;               // VGPU_GPU_CONCURRENCY: limited containers whose GPU-time
                                         // gates may be open together on one GPU (0 = any number;
                                         // -1 = "auto": 2 while the GPU's containers launch more than
                                         // pairs_on_rate kernels/s together, else any number)
  // VGPU_PAIRS_ON_RATE / VGPU_PAIRS_OFF_RATE: the "auto" thresholds. Three or more processes with
  // launches in flight each dispatch at about a quarter of the rate two reach (profiles/r6f): a
  // dispatch-bound crowd (4 LSTM pods: ~110k launches/s) gains from pairs, a compute-bound one
  // (16 ResNet-50 b=50 pods: ~16k/s) loses (profiles/r6k).
  uint32_t pairs_on_rate = 40000;
  uint32_t pairs_off_rate = 20000;
  int gpu_slice_ms = 20;                 // VGPU_GPU_SLICE_MS: turn length under that admission
  int cpu_node = -1;                     // VGPU_CPU_NODE (unless VGPU_CPU_SPREAD=0): the CPU node the
                                         // container's processes run on, published on the board
  bool use_ledger = true;                // VGPU_LEDGER: take charges from the node's GPU-time ledger
                                         // (vgpu/ledger.h) when its daemon keeps it fresh (the plugin
                                         // runs the daemon only with --ledger: profiles/r3v)
  int preempt_hold_ms = 3;               // VGPU_PREEMPT_HOLD_MS: background class - launches held while a
                                         // better class has waves on the GPU and this long after (0 = the
                                         // soft yield: only no credit is earned; profiles/r3s, r3t)
  int preempt_depth = 4;                 // VGPU_PREEMPT_DEPTH: background class - at most this many AQL
                                         // packets in flight per device while a better class shares the
                                         // GPU (0 = unbounded)
  int crowd_depth = 16;                  // VGPU_CROWD_DEPTH: on the GPU-time limiter of a crowded GPU, at
                                         // most this many AQL packets in flight per device and process, so
                                         // the credit gate acts per kernel instead of per queued batch
                                         // (0 = unbounded; 16 pods: slowest pod 0.96-1.01 of 1/N against
                                         // 0.79-0.99 unbounded, profiles/r5c)
  std::string lock_file = "/tmp/vgpulock/lock";  // host-PID discovery lock (reference /tmp/vgpulock/lock)
  int duplicate_merge = 1;               // merge two vGPUs of one physical GPU
  int duplicate_split = 0;               // VGPU_DUPLICATE_SPLIT: ... or keep them two devices (vdev_hooks.cpp)
  uint64_t host_mem_limit = 0;           // VGPU_HOST_MEMORY_LIMIT: pinned host memory, 0 = unlimited
  bool fail_open = false;                // VGPU_FAIL_OPEN: run unlimited when the region cannot be attached
  std::string device_map;                // VGPU_DEVICE_MAP ("<i>:<uuid> ...")
  std::string allowlist;                 // VGPU_ALLOWLIST: authorised GPU UUIDs, one per line ("" = no check)
  // Plugin-owned ceilings (limits file, see load_ceiling): the lowest task priority class the
  // container may take (VGPU_TASK_PRIORITY_MIN; 0 = latency class allowed) and the inode
  // of the region file the plugin created for it (VGPU_REGION_INODE, 0 = not checked).
  int min_priority = -1000;
  uint64_t region_inode = 0;
  bool ceiling = false;                  // a limits file was applied

  bool any_memory_limit() const;
  bool any_cu_limit() const;
};

// HBM reserve for small allocations under large-first spilling: the configured value, or
// max(min(2 GiB, hbm_share / 4), hbm_share / 16) — 18 GiB of a 288 GiB share, 512 MiB of 2 GiB.
uint64_t spill_reserve(const Config& cfg, uint64_t hbm_share);

// HBM a tenant with virtual device memory may hold above its HBM share for small allocations
// (below spill_small_bytes): RCCL transport buffers and tensors shared with DataLoader workers
// are exported over IPC, which a spilled (host-backed) buffer cannot be. The configured value,
// or min(1 GiB, hbm_share / 64) - 1 GiB of a 144 GiB share, 1 MiB of 64 MiB.
uint64_t spill_small_headroom(const Config& cfg, uint64_t hbm_share);

// Parses "NNN[KkMmGg][iB|B]" into bytes. Returns false on syntax error or overflow.
// Bare numbers are bytes; "m"/"M" is MiB, as in the reference ("<MiB>m").
bool parse_size(const char* s, uint64_t* out);

// Parses "<begin>-<end>" (end exclusive) or "<begin>:<count>".
bool parse_range(const char* s, int* begin, int* end);

// Fills `cfg` from the environment. `getenv_fn` is injectable for unit tests.
using GetenvFn = const char* (*)(const char*);
void load_config(Config* cfg, GetenvFn getenv_fn = nullptr);

// KEY=VALUE lines applied with setenv(…, overwrite=1) before the config is parsed
// (reference: nvml_preInit → load_env_from_file("/overrideEnv")).
int apply_override_env_file(const char* path);

// Plugin-owned limits (tamper resistance). The reference's limits come from container env
// and from a region the tenant maps read-write, and its set_current_device_memory_limit
// raises them from inside the container ([multiprocess_memory_limit.c:806-808]): a tenant
// can give itself more. Here the plugin also writes the container's contract into a limits
// file it owns, mounted read-only at kLimitsPath (docs/ABI.md). The shim treats it as the
// ceiling: the environment may only lower what it grants, and the device map, region path,
// compute-limit mode, oversubscription and the lowest priority class come from it.
constexpr const char* kLimitsPath = "/vgpu/limits";
// Parses a limits file (KEY=VALUE lines, the VGPU_* env names) into `out` (load_config
// semantics). False when it cannot be read.
bool load_ceiling(const char* path, Config* out);
// Clamps `cfg` (from the environment) to `ceil`.
void apply_ceiling(Config* cfg, const Config& ceil);
// Whether a limits file is present (kLimitsPath, or $VGPU_LIMITS_FILE): diagnostics
// switches that would turn enforcement off are then ignored.
bool ceiling_present();

// The process-wide config (filled by shim init).
const Config& config();
Config& mutable_config();

}  // namespace vgpu
