// Host waits on a crowded GPU: polling with short sleeps instead of the runtime's busy wait.
//
// Every HIP synchronisation (hipDeviceSynchronize - torch.cuda.synchronize -,
// hipStreamSynchronize, hipEventSynchronize) ends in ROCr's hsa_signal_wait_scacquire, which
// libamdhip64 imports. A GPU-bound PyTorch process spends its waits spinning on a CPU there
// (profiles/r4za: 1.1-1.6 CPUs busy per pod whatever the wait style, natively too). On a GPU
// shared by many pods that is one spinning core per pod doing nothing but wait for its turn:
// 16 pods of one GPU hold 16 cores, 128 on an 8-GPU node. The reference's throttle sleeps
// rather than spins (rate_limiter [multiprocess_utilization_watcher.c:53-72], nanosleep 10 ms).
//
// Here a blocking wait (HSA_WAIT_STATE_BLOCKED) - or an active one with a long time-out, the
// spin-until-done wait HIP uses when it schedules waits as "spin" (its default when the host
// has more cores than GPUs) - of a process whose GPU is crowded (the maintenance thread's
// crowd count: two or more other busy processes, watcher.cpp) becomes a loop of
// acquire-loads and nanosleeps; an active wait with a short time-out (HIP's brief spin before
// it blocks) stays as it is; the sleep grows with the time already waited (1/8 of
// it, 20 us to 500 us, after a 30 us spin that catches the short waits of tiny-kernel pods;
// the polling thread's timer slack is lowered to 1 us so a short sleep stays short), so a
// wait overshoots its completion by at most ~12 % (and 0.5 ms),
// and a multi-millisecond wait costs a few dozen wake-ups instead of a core. A lone pod, and
// a pod of the latency class (priority 0), keeps ROCr's own wait (no added latency);
// VGPU_SYNC_WAIT=poll|native forces either way.
#include <sys/prctl.h>
#include <time.h>

#include <algorithm>
#include <atomic>

#include "real.h"
#include "shim.h"
#include "vgpu/config.h"
#include "vgpu/ratelimit.h"

namespace vgpu {

std::atomic<uint64_t> g_sync_waits{0};      // blocking waits seen (VGPU_STATS)
std::atomic<uint64_t> g_sync_polled{0};     // of which polled
std::atomic<uint64_t> g_sync_wait_ns{0};    // time inside them
std::atomic<uint64_t> g_sync_wakeups{0};    // sleeps taken while polling
std::atomic<uint64_t> g_sync_active{0};     // active (spin-hinted) waits
std::atomic<uint64_t> g_sync_active_ns{0};

namespace {

// An active wait longer than this is a spin-until-done wait (HIP passes an unlimited
// time-out); shorter ones are the brief spin ahead of a blocking wait.
constexpr uint64_t kActiveSpinNs = 1'000'000;
// A polled wait spins this long before it sleeps.
constexpr uint64_t kPollSpinNs = 30'000;

// The polling thread's timer slack (Linux default 50 us, per thread) down to 1 us, once: a
// 20 us sleep then wakes after ~20 us instead of ~70 us.
void lower_timer_slack() {
  static thread_local bool done = false;
  if (done) return;
  done = true;
  (void)prctl(PR_SET_TIMERSLACK, 1000UL, 0, 0, 0);
}

bool satisfied(hsa_signal_condition_t c, hsa_signal_value_t v, hsa_signal_value_t cmp) {
  switch (c) {
    case HSA_SIGNAL_CONDITION_EQ: return v == cmp;
    case HSA_SIGNAL_CONDITION_NE: return v != cmp;
    case HSA_SIGNAL_CONDITION_LT: return v < cmp;
    case HSA_SIGNAL_CONDITION_GTE: return v >= cmp;
    default: return true;
  }
}

// Whether this process's waits should poll now. The latency class (task priority 0: a
// request-serving pod next to batch tenants) keeps ROCr's own wait - a polled wait may
// overshoot its completion by up to 1/8 of it, which such a pod's tail latency would pay;
// its one spinning core is the price of its class. Otherwise the device the wait is for
// decides: in a multi-GPU container, the calling thread's current HIP device (HIP's
// synchronisations wait in the calling thread), so a crowded GPU does not make the waits
// for an uncrowded one poll.
bool poll_now() {
  const SyncWait m = config().sync_wait;
  if (m == SyncWait::kPoll) return true;
  if (m == SyncWait::kNative) return false;
  ShimState& s = shim();
  if (!s.active || s.phase.load(std::memory_order_relaxed) != 2) return false;
  const Region* r = s.region.raw();
  if (effective_priority(r) <= 0) return false;
  bool any = false;
  for (int d = 0; d < s.n_agents; d++) any |= r->dev[d].crowd.load(std::memory_order_relaxed) > kAutoSpatialMaxCrowd;
  if (!any || s.n_agents == 1) return any;
  const int d = current_hip_agent();
  return d >= 0 && d < s.n_agents && r->dev[d].crowd.load(std::memory_order_relaxed) > kAutoSpatialMaxCrowd;
}

}  // namespace

}  // namespace vgpu

using namespace vgpu;

extern "C" {

hsa_signal_value_t hsa_signal_wait_scacquire(hsa_signal_t signal, hsa_signal_condition_t condition,
                                             hsa_signal_value_t compare_value, uint64_t timeout_hint,
                                             hsa_wait_state_t wait_state_hint) {
  VGPU_REAL_HSA(hsa_signal_wait_scacquire);
  const bool long_wait = wait_state_hint == HSA_WAIT_STATE_BLOCKED || timeout_hint > kActiveSpinNs;
  if (__builtin_expect(!long_wait || !poll_now(), 1)) {
    if (__builtin_expect(!g_stats_on, 1))
      return real_hsa_signal_wait_scacquire(signal, condition, compare_value, timeout_hint, wait_state_hint);
    const uint64_t t0 = now_ns();
    hsa_signal_value_t v =
        real_hsa_signal_wait_scacquire(signal, condition, compare_value, timeout_hint, wait_state_hint);
    const bool blocked = wait_state_hint == HSA_WAIT_STATE_BLOCKED;
    (blocked ? g_sync_waits : g_sync_active).fetch_add(1, std::memory_order_relaxed);
    (blocked ? g_sync_wait_ns : g_sync_active_ns).fetch_add(now_ns() - t0, std::memory_order_relaxed);
    return v;
  }
  VGPU_REAL_HSA(hsa_signal_load_scacquire);
  if (!real_hsa_signal_load_scacquire)
    return real_hsa_signal_wait_scacquire(signal, condition, compare_value, timeout_hint, wait_state_hint);
  const uint64_t t0 = now_ns();
  hsa_signal_value_t v = real_hsa_signal_load_scacquire(signal);
  uint64_t wakeups = 0;
  // A short spin first: a pod that waits every few tiny kernels would otherwise pay a sleep's
  // wake-up latency on every wait (profiles/r6a3: 8-kernel waits capped at ~40k kernels/s).
  while (!satisfied(condition, v, compare_value) && now_ns() - t0 < kPollSpinNs) {
    __builtin_ia32_pause();
    v = real_hsa_signal_load_scacquire(signal);
  }
  if (!satisfied(condition, v, compare_value)) lower_timer_slack();
  while (!satisfied(condition, v, compare_value)) {
    const uint64_t el = now_ns() - t0;
    if (el >= timeout_hint) break;
    const uint64_t sl = std::min<uint64_t>(std::max<uint64_t>(el / 8, 20'000), 500'000);
    struct timespec ts = {0, (long)std::min<uint64_t>(sl, timeout_hint - el)};
    nanosleep(&ts, nullptr);
    wakeups++;
    v = real_hsa_signal_load_scacquire(signal);
  }
  if (__builtin_expect(g_stats_on, 0)) {
    g_sync_waits.fetch_add(1, std::memory_order_relaxed);
    g_sync_polled.fetch_add(1, std::memory_order_relaxed);
    g_sync_wait_ns.fetch_add(now_ns() - t0, std::memory_order_relaxed);
    g_sync_wakeups.fetch_add(wakeups, std::memory_order_relaxed);
  }
  return v;
}

}  // extern "C"
