/* C ABI over the shared region, for the node monitor, vgpuctl and tests.
 *
 * Reference: the shim's exported control functions (suspend_all@[870],
 * resume_all@[878], set_current_device_sm_limit_scale [787-789],
 * set_current_device_memory_limit [806-808], get_current_device_* [798-842]),
 * which an external monitor reached by loading libvgpu.so. Here the same
 * operations are exposed on an explicit region handle from a library that does
 * not interpose anything (libvgpu_region.so), plus process-local variants exported
 * by the shim itself (vgpu_self_*). */
#ifndef VGPU_REGION_API_H
#define VGPU_REGION_API_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct vgpu_region vgpu_region;

typedef struct {
  int32_t pid;
  int32_t hostpid;
  int32_t status;
  int32_t priority;
  uint64_t launches;
  uint64_t throttle_ns;
  uint64_t suspend_ns;
  uint64_t oom_events;
  uint64_t used[16];
  uint64_t used_kind[16][4];
  uint64_t peak[16];
  uint64_t host_used;  /* pinned host memory */
  uint64_t host_peak;
} vgpu_proc_info;

typedef struct {
  char uuid[64];
  uint64_t mem_limit;
  uint64_t phys_total;
  uint64_t used;
  uint64_t spilled;
  uint64_t monitor_used;
  int32_t cu_limit_pct;
  int32_t cu_count;
  int32_t num_xcc;
  int32_t cu_mask_count;
  uint32_t cu_mask[8];
  int64_t credit_ns;   /* temporal mode: remaining GPU-time credit */
  uint64_t charged_ns; /* GPU time charged to the container */
  uint64_t wall_ns;    /* wall time accounted by the sampler */
  int32_t util_pct;    /* smoothed utilisation (charged / wall), percent */
  int32_t cu_mode;     /* effective mode: 0 off, 1 spatial, 2 temporal, 3 both */
  uint32_t gpu_id;
  uint32_t bdf;
  uint32_t domain;
  uint32_t configured;
  uint64_t hbm_limit;
  int32_t crowd;       /* auto mode: other busy processes seen on the GPU (-1 = not assessed) */
  int32_t preempt;     /* background class: launches held, a better class is busy (1) */
  int32_t depth_cap;   /* background class: packets in flight allowed per process (0 = any) */
  int32_t cu_share_bp; /* exact GPU-time share of the grants, basis points (0 = cu_limit_pct) */
} vgpu_device_info;

/* Returns NULL on failure; *err receives -errno. */
vgpu_region* vgpu_region_open(const char* path, int create, int* err);
void vgpu_region_close(vgpu_region* r);
uint32_t vgpu_region_version(void);
uint64_t vgpu_region_size(void);
int vgpu_region_num_devices(vgpu_region* r);
int vgpu_region_device_info(vgpu_region* r, int dev, vgpu_device_info* out);
int vgpu_region_proc_count(vgpu_region* r);
/* Fills up to `max` live process records; returns the number written. */
int vgpu_region_procs(vgpu_region* r, vgpu_proc_info* out, int max);
int vgpu_region_set_memory_limit(vgpu_region* r, int dev, uint64_t bytes);
int vgpu_region_set_cu_limit(vgpu_region* r, int dev, int pct);
/* Sets the exact GPU-time share (basis points, 0 = the whole-percent limit) as it stands in
   the region: what a container's limiter grants from (a plugin ceiling clamps it). */
int vgpu_region_set_cu_share(vgpu_region* r, int dev, int bp);
/* Sets the HBM-resident share of an oversubscribed vGPU (0 = no cap; a plugin ceiling clamps it). */
int vgpu_region_set_hbm_limit(vgpu_region* r, int dev, uint64_t bytes);
int vgpu_region_suspend_all(vgpu_region* r);
int vgpu_region_resume_all(vgpu_region* r);
int vgpu_region_suspended(vgpu_region* r);
int vgpu_region_set_priority(vgpu_region* r, int prio);
int vgpu_region_get_priority(vgpu_region* r);
int vgpu_region_set_recent_kernel(vgpu_region* r, int v);
int vgpu_region_get_recent_kernel(vgpu_region* r);
int vgpu_region_set_utilization_switch(vgpu_region* r, int v);
/* Occupancy-sampler ticks so far (temporal mode; the sampling rate over a window). */
uint64_t vgpu_region_samples(vgpu_region* r);
/* Of those, the ticks that re-read the other processes' occupancy (crowd-stretched). */
uint64_t vgpu_region_other_refreshes(vgpu_region* r);
int vgpu_region_reclaim(vgpu_region* r);
/* Pinned host memory of the container: limit (0 = unlimited) and aggregate usage. */
int vgpu_region_host_info(vgpu_region* r, uint64_t* limit, uint64_t* used);
int vgpu_region_set_host_limit(vgpu_region* r, uint64_t bytes);
int vgpu_region_charge_host(vgpu_region* r, int slot, uint64_t bytes);
void vgpu_region_uncharge_host(vgpu_region* r, int slot, uint64_t bytes);
/* Test hooks: charge/uncharge through the same admission path the shim uses. */
int vgpu_region_register(vgpu_region* r, int32_t pid, int32_t hostpid);
void vgpu_region_unregister(vgpu_region* r, int slot);
int vgpu_region_charge(vgpu_region* r, int slot, int dev, uint64_t bytes, int kind);
void vgpu_region_uncharge(vgpu_region* r, int slot, int dev, uint64_t bytes, int kind);
/* CU-mask helpers (same code the shim uses). */
int vgpu_cu_share_count(int cu_count, int num_xcc, int pct);
void vgpu_cu_partition_range(int cu_count, int num_xcc, int split, int slot, int* begin, int* end);
/* Env parsing helper: bytes or -1. */
int64_t vgpu_parse_size(const char* s);

#ifdef __cplusplus
}
#endif
#endif
