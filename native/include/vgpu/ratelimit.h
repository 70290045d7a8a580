// Temporal compute limiter: a GPU-time credit per container and device.
//
// Reference: libvgpu.so src/multiprocess/multiprocess_utilization_watcher.c
//   rate_limiter [53-72]  tokens = grid blocks; spin while recent_kernel < 0;
//                         CAS tokens -= grids; while tokens < 0 sleep 10 ms
//   delta@0x46712         proportional controller on |limit - util|
//   utilization_watcher   every 120 ms: sample NVML SM util, share = delta(...),
//                         tokens = min(tokens + share, total)
//
// The reference prices a launch in grid blocks and steers the refill from a 120 ms
// utilisation sample, so the achieved share depends on kernel shapes (a workgroup of a
// 2 µs kernel costs the same as one of a 2 ms kernel) and the loop oscillates. Round 1
// kept that structure and measured 29/44/62 % for 25/50/75 % limits.
//
// MI355X design: the currency is GPU time itself.
//   * A sampler (one elected process per container) reads KFD's per-process
//     cu_occupancy for the container's host PIDs and for every other process on the
//     same GPU every ~1 ms (a read costs ~29 µs, profiles/r2a/occ_probe.json). While the
//     container has resident waves it is charged the wall time of the interval,
//     weighted by its share of all resident waves on the GPU (processor-sharing: when
//     k tenants run concurrently each gets about 1/k of the throughput, and is charged
//     1/k of the time). Alone on the GPU it is charged exactly its busy time.
//   * Each interval also grants limit% of the wall time. credit = grants − charges,
//     clamped to [-debt, +burst].
//   * The launch gate (every kernel / graph launch) passes while credit > 0 and sleeps
//     otherwise. Work already queued on the GPU keeps running and keeps being charged,
//     so the credit goes into debt and the gate stays closed until the debt is repaid:
//     the long-run busy fraction converges to limit% regardless of launch granularity
//     or queue depth.
// No tokens are priced per launch; the launch path is one relaxed load.
#pragma once

#include <cstdint>

#include "vgpu/region.h"

namespace vgpu {

struct TimeShareParams {
  int limit_pct = 100;       // 0 or >= 100 = unlimited
  int limit_bp = 0;          // exact share in basis points (0 = limit_pct)
  int64_t burst_ns = 0;      // positive credit cap
  int64_t debt_ns = 0;       // negative credit floor (as a positive number)
  int64_t reopen_ns = 0;     // a closed gate re-opens once the credit reaches this
};

// Default clamps for a limit: burst = max(4 ms, limit% of `window_ms`, default 40 ms),
// re-open threshold burst / 2, debt = 2 s. The hysteresis makes on/off periods several milliseconds
// long instead of one sample: every restart after an idle gap costs the tenant some
// throughput (clocks and caches ramp up again), so fewer, longer periods track the
// limit more closely (profiles/r2b vs r2c).
TimeShareParams timeshare_params(int limit_pct, int window_ms = 40, int limit_bp = 0);

// Gate state after a sample: an open gate stays open while credit > 0; a closed gate
// re-opens once credit >= reopen_ns.
inline bool timeshare_gate(bool open, int64_t credit, const TimeShareParams& p) {
  return open ? credit > 0 : credit >= p.reopen_ns;
}

// Charge for `dt_ns` of wall time in which the container held `mine` of the `total`
// resident waves (CUs' worth) on the device. mine <= 0 → 0; total < mine → total = mine.
int64_t timeshare_charge(int64_t dt_ns, int64_t mine, int64_t total);

// Progress-floor charge fraction (per mille) of a sample: the share `share_pm`, raised to
// the container's occupancy relative to `ref` - its own recent peak occupancy, i.e. what
// it holds when nothing slows it down. Tenants that co-run without losing occupancy (two
// light inference pods) then pay what they would pay alone instead of 1/k of it each;
// tenants that crowd each other out (occupancy drops to ~1/k of the peak) pay their
// share as before. Alone, the share is already 1000.
int timeshare_progress_pm(int share_pm, int64_t mine, int64_t ref);

// Decaying peak of a container's occupancy: max(mine, ref - ref/2048) per sample (a
// half-life of ~1400 samples, seconds at the sampler's rate).
inline int64_t occupancy_ref_update(int64_t ref, int64_t mine) {
  const int64_t decayed = ref - (ref >> 11);
  return mine > decayed ? mine : decayed;
}

// GPU time of an interval estimated from the charge fractions (per mille, 0..1000) at
// its two end samples: trapezoid rule, except that an interval which began with the
// gate re-opening (credit crossed above zero at the previous sample, so the container's
// work resumed right after it) and started idle is charged at the end-point rate. The
// plain end-point rule misses half an interval at every busy→idle edge; the trapezoid
// alone misses half of one at every gate-triggered start (simulated in core_tests.cpp).
int64_t timeshare_interval(int64_t dt_ns, int prev_pm, int now_pm, bool gate_opened_at_prev);

// One accounting step: credit + grant_dt*limit/100 − charge, clamped. Pure. `grant_dt`
// is the part of the interval that earns credit (dt, or 0 while a background tenant
// yields; < 0 = dt).
int64_t timeshare_step(int64_t credit, const TimeShareParams& p, int64_t dt_ns, int64_t charge_ns,
                       int64_t grant_dt_ns = -1);

// Applies one step to the region's device state (credit, gate, cumulative charged time
// and the smoothed utilisation shown by vgpuctl / the monitor).
void timeshare_apply(DeviceState& d, const TimeShareParams& p, int64_t dt_ns, int64_t charge_ns,
                     int64_t grant_dt_ns = -1);

// Launch-side gate. Blocks while the region's launch block is set (recent_kernel < 0,
// every cu mode) and, when `limited`, while the device's credit is exhausted and the
// sampler is alive. Returns nanoseconds spent blocked. `poll_ns` is the back-off.
uint64_t limiter_acquire(RegionHeader& h, DeviceState& d, bool limited, int64_t poll_ns = 200'000);

// True if the launch block or an exhausted credit would make limiter_acquire wait.
inline bool limiter_would_block(const RegionHeader& h, const DeviceState& d, bool limited) {
  return h.recent_kernel.load(std::memory_order_relaxed) < 0 ||
         (limited && !d.gate_open.load(std::memory_order_relaxed));
}

// Occupancy sampling period on a crowded GPU. Every limited container samples its own
// processes and every other process on the GPU, and each KFD cu_occupancy read walks the
// GPU's wave slots (~29 µs, profiles/r2a): with n processes the node reads about n² files
// per period. Sampling everything every 1 ms cost 12 pods 14 % of the GPU (0.86x
// aggregate); every ~4.5 ms, 2-6 % (0.94-0.98x, profiles/r2ae, r2af, r2ag). Re-reading
// only the pod's own processes every 1 ms and the others every ~4.5 ms measured 0.85x
// (profiles/r2aj): part of the gain comes from the coarser gate decisions themselves
// (longer on/off periods, fewer restarts). The period covering `reads` node-wide reads
// (n² here) stretches to base·reads/budget once reads > budget, at most `max_ns`.
inline int64_t sample_period_ns(int64_t base_ns, int64_t reads, int budget, int64_t max_ns) {
  if (budget <= 0 || reads <= budget) return base_ns;
  int64_t p = base_ns * reads / budget;
  return p < max_ns ? p : (max_ns > base_ns ? max_ns : base_ns);
}

uint64_t now_ns();

}  // namespace vgpu
