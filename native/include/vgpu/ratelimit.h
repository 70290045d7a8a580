// Temporal compute limiter (reference-parity mode).
//
// Reference: libvgpu.so src/multiprocess/multiprocess_utilization_watcher.c
//   rate_limiter [53-72]  tokens = grid blocks; spin while recent_kernel < 0;
//                         CAS tokens -= grids; while tokens < 0 sleep 10 ms
//   delta@0x46712         proportional controller on |limit - util|
//   utilization_watcher   every 120 ms: sample util, share = delta(...),
//                         tokens = min(tokens + share, total)
//
// Differences: the bucket lives in the shared region (one budget per container and
// device, not one per process) and one elected process runs the watcher. The
// reference's controller steps by a chip-size constant (sm^2 * maxThreads * diff /
// 2560) into a bucket of sm * maxThreads * 32 tokens, so a tenant runs unthrottled
// until millions of workgroups have drained the initial bucket and then oscillates.
// Here the refill `share` is adjusted relative to itself (proportional decrease to
// limit/util, multiplicative increase by the headroom) and the bucket holds two
// periods' worth, so the duty cycle converges within a few 120 ms periods.
#pragma once

#include <cstdint>

#include "vgpu/region.h"

namespace vgpu {

struct LimiterSpec {
  int cu_count = 256;
  int max_threads_per_cu = 2048;  // 32 waves x 64 lanes
  // Upper bound of the per-period share (the reference's g_total_cuda_cores).
  int64_t total() const { return (int64_t)cu_count * max_threads_per_cu * 32; }
  // One full wave of single-wave workgroups on the chip.
  int64_t wave() const { return (int64_t)cu_count * (max_threads_per_cu / 64); }
  // Minimum share: one workgroup per CU per period, so a tenant is never starved.
  int64_t floor() const { return cu_count > 0 ? cu_count : 1; }
};

// Starting share (and bucket) for a limit: limit% of one chip wave.
int64_t limiter_initial_share(const LimiterSpec& spec, int limit_pct);

// One controller step: returns the new per-period refill `share`.
int64_t limiter_delta(const LimiterSpec& spec, int limit_pct, int util_pct, int64_t share);

// Periodic refill after a utilisation sample: share = delta(...), cap = 2 * share,
// tokens = min(tokens + share, cap).
void limiter_refill(DeviceState& d, const LimiterSpec& spec, int limit_pct, int util_pct);

// Blocking token acquisition for a launch of `workgroups` on device state `d`.
// Returns nanoseconds spent waiting. `sleep_ns` is the back-off (reference: 10 ms).
uint64_t limiter_acquire(RegionHeader& h, DeviceState& d, int64_t workgroups, int64_t sleep_ns = 10'000'000);

uint64_t now_ns();

}  // namespace vgpu
