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
// device, not one per process), one elected process runs the watcher, and the
// controller constants are derived from the MI355X agent (CUs x max threads per CU).
#pragma once

#include <cstdint>

#include "vgpu/region.h"

namespace vgpu {

struct LimiterSpec {
  int cu_count = 256;
  int max_threads_per_cu = 2048;  // 32 waves x 64 lanes
  int64_t total() const { return (int64_t)cu_count * max_threads_per_cu * 32; }
};

// One controller step: returns the new per-period refill `share`.
int64_t limiter_delta(const LimiterSpec& spec, int limit_pct, int util_pct, int64_t share);

// Periodic refill after a utilisation sample. Implements the reference's
// "if share == total and tokens < 0, double total" escape for very large grids.
void limiter_refill(DeviceState& d, const LimiterSpec& spec, int limit_pct, int util_pct);

// Blocking token acquisition for a launch of `workgroups` on device state `d`.
// Returns nanoseconds spent waiting. `sleep_ns` is the back-off (reference: 10 ms).
uint64_t limiter_acquire(RegionHeader& h, DeviceState& d, int64_t workgroups, int64_t sleep_ns = 10'000'000);

uint64_t now_ns();

}  // namespace vgpu
