// KFD sysfs helpers: host-PID discovery and per-process GPU usage signals.
//
// Reference: set_task_pid [src/utils.c:188-255] diffs NVML's running-process list
// around cuDevicePrimaryCtxRetain, under the "unified lock" /tmp/vgpulock/lock
// (try_lock_unified_lock [utils.c:30-36]), to learn the process's host PID (NVML
// reports host PIDs, the container sees namespaced ones); the utilisation watcher
// retries it while it is unknown (update_host_pid [multiprocess_utilization_watcher.c:
// 195-216]).
//
// On MI355X the KFD exposes /sys/class/kfd/kfd/proc/<host-pid>/ for every process that
// opened /dev/kfd. sysfs is not PID-namespaced, but it is node-wide: on a busy node
// processes of other containers (other GPUs included) appear and vanish all the time,
// so a before/after diff is ambiguous (measured on the gpurun box: 3 of 4 concurrent
// starters unresolved, profiles/r2a/occ_probe.json). The resolution here is a VRAM
// signature instead: allocate a buffer of an unusual size and pick the KFD process
// whose vram_<gpu_id> grew by exactly that much; confirm with a second size.
//
// The same tree carries stats_<gpu_id>/cu_occupancy (CUs' worth of resident waves),
// the utilisation signal of the temporal limiter (the reference uses
// nvmlDeviceGetProcessUtilization).
#pragma once

#include <sys/types.h>

#include <cstdint>
#include <vector>

namespace vgpu {

extern const char* g_kfd_proc_root;  // overridable for tests

std::vector<int> kfd_list_pids();
// New PIDs in `after` that were not in `before`; returns the unique one or 0.
pid_t kfd_diff_pid(const std::vector<int>& before, const std::vector<int>& after);
// cu_occupancy of hostpid on KFD gpu_id, -1 if unreadable.
int64_t kfd_cu_occupancy(pid_t hostpid, uint32_t gpu_id);
// VRAM bytes charged by KFD to hostpid on gpu_id (vram_<gpu_id>), -1 if unreadable.
int64_t kfd_vram_usage(pid_t hostpid, uint32_t gpu_id);
// Host PIDs that have a queue-statistics directory for gpu_id (i.e. use that GPU).
std::vector<int> kfd_pids_on_gpu(uint32_t gpu_id);

// Allocates (alloc = true) or frees `bytes` of device memory on the GPU through the
// real allocator, outside any quota. Returns false when the allocation failed.
using VramProbe = bool (*)(void* ctx, uint64_t bytes, bool alloc);

// Resolves this process's host PID. Returns getpid() when KFD lists it (no PID
// namespace); otherwise runs the VRAM-signature search over `probe` while holding an
// exclusive flock on `lock_path` (created if missing; null = no lock; waits at most
// `lock_timeout_ms`). Returns 0 when unresolved (the caller retries later).
pid_t kfd_resolve_hostpid(uint32_t gpu_id, VramProbe probe, void* ctx, const char* lock_path,
                          int lock_timeout_ms, unsigned seed);

// Exclusive flock on `path`, polling up to timeout_ms. An existing file is opened
// read-only (the plugin mounts it so); a missing one is created, world-accessible.
// Returns the fd (release with kfd_unlock), kLockBusy when another holder kept it for the
// whole wait, or kLockUnavailable when the file cannot be opened.
constexpr int kLockBusy = -2;
constexpr int kLockUnavailable = -1;
int kfd_lock(const char* path, int timeout_ms);
void kfd_unlock(int fd);

}  // namespace vgpu
