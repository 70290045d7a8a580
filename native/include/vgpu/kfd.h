// KFD sysfs helpers: host-PID discovery and per-process CU occupancy.
//
// Reference: set_task_pid [src/utils.c:188-255] diffs NVML's running-process list
// around cuDevicePrimaryCtxRetain to learn the process's host PID (NVML reports
// host PIDs, the container sees namespaced ones). On MI355X the KFD exposes
// /sys/class/kfd/kfd/proc/<host-pid>/ for every process that opened /dev/kfd;
// sysfs is not PID-namespaced, so diffing that directory around hsa_init gives the
// same answer without a vendor library. The same tree carries
// stats_<gpu_id>/cu_occupancy (CUs' worth of resident waves), which is the
// per-process utilisation signal for the temporal limiter (the reference uses
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

}  // namespace vgpu
