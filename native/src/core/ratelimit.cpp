#include "vgpu/ratelimit.h"

#include <time.h>

#include <algorithm>

namespace vgpu {

uint64_t now_ns() {
  struct timespec ts;
  clock_gettime(CLOCK_MONOTONIC, &ts);
  return (uint64_t)ts.tv_sec * 1000000000ull + (uint64_t)ts.tv_nsec;
}

TimeShareParams timeshare_params(int limit_pct, int window_ms, int limit_bp) {
  TimeShareParams p;
  p.limit_pct = limit_pct;
  const bool limited = limit_pct > 0 && limit_pct < 100;
  p.limit_bp = limited && limit_bp > 0 && limit_bp < 10000 ? limit_bp : 0;
  const int64_t bp = p.limit_bp ? p.limit_bp : (limited ? limit_pct : 100) * 100;
  if (window_ms <= 0) window_ms = 40;
  p.burst_ns = std::max<int64_t>(4'000'000, (int64_t)window_ms * 1'000'000ll * bp / 10000);
  p.reopen_ns = p.burst_ns / 2;
  p.debt_ns = 2'000'000'000ll;
  return p;
}

int64_t timeshare_charge(int64_t dt_ns, int64_t mine, int64_t total) {
  if (dt_ns <= 0 || mine <= 0) return 0;
  if (total < mine) total = mine;
  // 128-bit free: dt (< 2^40 for any sane interval) * mine (<= a few thousand waves).
  return dt_ns * mine / total;
}

int timeshare_progress_pm(int share_pm, int64_t mine, int64_t ref) {
  if (mine <= 0 || ref <= 0) return share_pm;
  const int64_t rel = mine >= ref ? 1000 : mine * 1000 / ref;
  return rel > share_pm ? (int)rel : share_pm;
}

int64_t timeshare_interval(int64_t dt_ns, int prev_pm, int now_pm, bool gate_opened_at_prev) {
  if (dt_ns <= 0) return 0;
  if (gate_opened_at_prev && prev_pm == 0) return dt_ns * now_pm / 1000;
  return dt_ns * (prev_pm + now_pm) / 2000;
}

int64_t timeshare_step(int64_t credit, const TimeShareParams& p, int64_t dt_ns, int64_t charge_ns,
                       int64_t grant_dt_ns) {
  if (dt_ns < 0) dt_ns = 0;
  if (grant_dt_ns < 0 || grant_dt_ns > dt_ns) grant_dt_ns = dt_ns;
  const int64_t bp = p.limit_bp > 0 ? p.limit_bp : (p.limit_pct > 0 && p.limit_pct < 100 ? p.limit_pct : 100) * 100;
  credit += grant_dt_ns * bp / 10000 - charge_ns;
  if (credit > p.burst_ns) credit = p.burst_ns;
  if (credit < -p.debt_ns) credit = -p.debt_ns;
  return credit;
}

void timeshare_apply(DeviceState& d, const TimeShareParams& p, int64_t dt_ns, int64_t charge_ns,
                     int64_t grant_dt_ns) {
  // Single writer (the sampler lease holder); launch gates only read the credit.
  int64_t c = timeshare_step(d.credit_ns.load(std::memory_order_relaxed), p, dt_ns, charge_ns, grant_dt_ns);
  d.credit_ns.store(c, std::memory_order_release);
  d.gate_open.store(timeshare_gate(d.gate_open.load(std::memory_order_relaxed) != 0, c, p) ? 1 : 0,
                    std::memory_order_release);
  d.charged_ns.fetch_add((uint64_t)std::max<int64_t>(0, charge_ns), std::memory_order_relaxed);
  d.wall_ns.fetch_add((uint64_t)std::max<int64_t>(0, dt_ns), std::memory_order_relaxed);
  // Utilisation over roughly the last 100 ms (EWMA of the charged fraction, per mille).
  if (dt_ns > 0) {
    int64_t frac = std::min<int64_t>(1000, charge_ns * 1000 / dt_ns);
    int64_t prev = d.util_pm.load(std::memory_order_relaxed);
    int64_t alpha = std::min<int64_t>(1000, dt_ns / 100'000);  // dt / 100 ms, per mille
    d.util_pm.store((int32_t)(prev + (frac - prev) * alpha / 1000), std::memory_order_relaxed);
  }
}

uint64_t limiter_acquire(RegionHeader& h, DeviceState& d, bool limited, int64_t poll_ns) {
  uint64_t t0 = 0;
  struct timespec ts = {(time_t)(poll_ns / 1000000000), (long)(poll_ns % 1000000000)};
  // External launch block (reference: recent_kernel < 0), honoured in every cu mode.
  while (h.recent_kernel.load(std::memory_order_relaxed) < 0) {
    if (!t0) t0 = now_ns();
    nanosleep(&ts, nullptr);
  }
  while (limited && !d.gate_open.load(std::memory_order_acquire)) {
    if (!t0) t0 = now_ns();
    // Without a live sampler nobody repays the debt: never block forever. The same when
    // the device left the GPU-time limiter while this launch waited (cu_mode bit 2).
    uint64_t hb = h.watcher_heartbeat.load(std::memory_order_relaxed);
    if (!hb || now_ns() - hb > 1'000'000'000ull) break;
    if (!(d.cu_mode.load(std::memory_order_relaxed) & 2)) break;
    nanosleep(&ts, nullptr);
  }
  return t0 ? now_ns() - t0 : 0;
}

}  // namespace vgpu
