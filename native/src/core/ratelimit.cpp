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
  const int64_t total = spec.total();
  int64_t diff = std::abs(limit_pct - util_pct);
  if (diff < 5) diff = 5;
  int64_t inc = (int64_t)spec.cu_count * spec.cu_count * spec.max_threads_per_cu * diff / 2560;
  if (diff > limit_pct / 2) inc = inc * diff * 2 / (limit_pct + 1);
  if (util_pct < limit_pct) share = std::min(share + inc, total);
  else share = std::max<int64_t>(share - inc, 0);
  return share;
}

void limiter_refill(DeviceState& d, const LimiterSpec& spec, int limit_pct, int util_pct) {
  int64_t cap = d.token_cap.load();
  if (cap <= 0) cap = spec.total();
  int64_t share = d.share.load();
  int64_t tokens = d.tokens.load();
  if (share >= cap && tokens < 0) cap *= 2;  // grids larger than the bucket
  share = limiter_delta(spec, limit_pct, util_pct, share);
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
