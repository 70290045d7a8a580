#include "vgpu/ratelimit.h"

#include <time.h>

#include <algorithm>
#include <cstdlib>

namespace vgpu {

uint64_t now_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

int64_t limiter_delta(const LimiterSpec& spec, int limit_pct, int util_pct, int64_t share) {
  const int64_t floor = spec.floor();
  const int64_t ceil = spec.total();
  if (share < floor) share = floor;
  if (util_pct > limit_pct) {
    // Proportional decrease toward limit/util, at most halving per period.
    int64_t num = std::max(limit_pct, util_pct / 2);
    share = std::max(floor, share * num / std::max(util_pct, 1));
  } else if (util_pct < limit_pct) {
    // Proportional increase toward limit/util (at most 4x per period), so a saturating
    // tenant reaches its share in a handful of 120 ms periods instead of ramping +50 %
    // at a time; an idle tenant (util 0) grows 1.5x plus one wave.
    if (util_pct > 0) {
      int64_t num = std::min<int64_t>(limit_pct, 4 * (int64_t)util_pct);
      share = std::min(ceil, std::max(share + floor, share * num / util_pct));
    } else {
      share = std::min(ceil, share + share / 2 + floor);
    }
  }
  return share;
}

int64_t limiter_initial_share(const LimiterSpec& spec, int limit_pct) {
  int64_t pct = limit_pct > 0 && limit_pct < 100 ? limit_pct : 100;
  return std::max(spec.floor(), spec.wave() * pct / 100);
}

void limiter_refill(DeviceState& d, const LimiterSpec& spec, int limit_pct, int util_pct) {
  int64_t share = limiter_delta(spec, limit_pct, util_pct, d.share.load());
  // Burst capacity of two periods: small enough that a saturating tenant is throttled
  // within ~2 periods of exceeding its share; grids larger than the bucket simply
  // wait for several refills (tokens go negative, never deadlock).
  int64_t cap = 2 * share;
  d.share.store(share);
  d.token_cap.store(cap);
  d.util_pct.store(util_pct);
  int64_t cur = d.tokens.load();
  while (!d.tokens.compare_exchange_weak(cur, std::min(cur + share, cap))) {
  }
}

uint64_t limiter_acquire(RegionHeader& h, DeviceState& d, int64_t workgroups, int64_t sleep_ns) {
  uint64_t waited = 0;
  uint64_t t0 = 0;
  struct timespec ts = {(time_t)(sleep_ns / 1000000000), (long)(sleep_ns % 1000000000)};
  // External launch block (reference: recent_kernel < 0).
  while (h.recent_kernel.load(std::memory_order_relaxed) < 0) {
    if (!t0) t0 = now_ns();
    nanosleep(&ts, nullptr);
  }
  if (h.recent_kernel.load(std::memory_order_relaxed) != 2) h.recent_kernel.store(2, std::memory_order_relaxed);
  d.tokens.fetch_sub(workgroups, std::memory_order_acq_rel);
  while (d.tokens.load(std::memory_order_acquire) < 0) {
    if (!t0) t0 = now_ns();
    // If no watcher refills (it died and nobody took over yet) do not block forever.
    uint64_t hb = h.watcher_heartbeat.load(std::memory_order_relaxed);
    if (hb && now_ns() - hb > 2'000'000'000ull) break;
    nanosleep(&ts, nullptr);
  }
  if (t0) waited = now_ns() - t0;
  return waited;
}

}  // namespace vgpu
