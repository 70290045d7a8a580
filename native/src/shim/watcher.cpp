// Utilisation watcher: the feedback loop of the temporal limiter, plus the
// monitor-based memory accounting and the active OOM killer.
//
// Reference: utilization_watcher@0x471a7 [multiprocess_utilization_watcher.c:195-216]
// samples NVML per-process SM utilisation every 120 ms, sums it over the region's
// host PIDs, refills the token bucket through delta(), and feeds
// set_gpu_device_memory_monitor → active_oom_killer (SIGKILL every region process).
//
// MI355X: the signal is KFD's per-process cu_occupancy (CUs' worth of resident
// waves), sampled several times per period and averaged; fallback is the device's
// gpu_busy_percent. One process per region holds the watcher lease (watcher_pid +
// heartbeat) so the container has a single controller and a single bucket. The OOM
// killer terminates the largest consumer instead of every process.
#include <dirent.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <cstdio>
#include <cstring>

#include "shim.h"
#include "vgpu/kfd.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

namespace vgpu {

namespace {

// Device-wide busy percent for KFD gpu_id via the topology's render minor.
int device_busy_percent(uint32_t gpu_id) {
  static char cached_path[kMaxDevices][128];
  static uint32_t cached_id[kMaxDevices];
  int slot = -1;
  for (int i = 0; i < kMaxDevices; i++) {
    if (cached_id[i] == gpu_id && cached_path[i][0]) {
      slot = i;
      break;
    }
  }
  if (slot < 0) {
    DIR* d = opendir("/sys/class/kfd/kfd/topology/nodes");
    if (!d) return -1;
    int minor = -1;
    while (struct dirent* e = readdir(d)) {
      if (e->d_name[0] == '.') continue;
      char p[512];
      snprintf(p, sizeof(p), "/sys/class/kfd/kfd/topology/nodes/%s/gpu_id", e->d_name);
      FILE* f = fopen(p, "r");
      if (!f) continue;
      unsigned id = 0;
      bool ok = fscanf(f, "%u", &id) == 1;
      fclose(f);
      if (!ok || id != gpu_id) continue;
      snprintf(p, sizeof(p), "/sys/class/kfd/kfd/topology/nodes/%s/properties", e->d_name);
      f = fopen(p, "r");
      if (!f) continue;
      char key[64];
      long long val;
      while (fscanf(f, "%63s %lld", key, &val) == 2)
        if (!strcmp(key, "drm_render_minor")) minor = (int)val;
      fclose(f);
    }
    closedir(d);
    if (minor < 0) return -1;
    for (int i = 0; i < kMaxDevices; i++) {
      if (!cached_path[i][0]) {
        snprintf(cached_path[i], sizeof(cached_path[i]), "/sys/class/drm/renderD%d/device/gpu_busy_percent", minor);
        cached_id[i] = gpu_id;
        slot = i;
        break;
      }
    }
    if (slot < 0) return -1;
  }
  FILE* f = fopen(cached_path[slot], "r");
  if (!f) return -1;
  int v = -1;
  if (fscanf(f, "%d", &v) != 1) v = -1;
  fclose(f);
  return v;
}

bool take_lease(Region* r, pid_t me) {
  int32_t cur = r->hdr.watcher_pid.load();
  if (cur == me) return true;
  uint64_t hb = r->hdr.watcher_heartbeat.load();
  bool stale = cur == 0 || kill(cur, 0) != 0 || (hb && now_ns() - hb > 1'000'000'000ull);
  if (!stale) return false;
  return r->hdr.watcher_pid.compare_exchange_strong(cur, me);
}

void* watcher_main(void*) {
  ShimState& s = shim();
  Region* r = s.region.raw();
  const Config& cfg = config();
  const int period_ms = cfg.util_period_ms;
  const int samples = 6;
  struct timespec tick = {0, (long)period_ms * 1000000L / samples};
  pid_t me = getpid();
  while (!s.exiting.load() && s.pid == me) {
    if (!take_lease(r, me)) {
      struct timespec ts = {0, (long)period_ms * 1000000L};
      nanosleep(&ts, nullptr);
      continue;
    }
    int64_t occ_sum[kMaxDevices] = {0};
    int occ_ok[kMaxDevices] = {0};
    for (int k = 0; k < samples; k++) {
      for (int d = 0; d < s.n_agents; d++) {
        if (!s.agents[d].gpu_id) continue;
        int64_t sum = 0;
        bool any = false;
        for (int i = 0; i < kMaxProcs; i++) {
          if (!r->procs[i].pid.load(std::memory_order_relaxed)) continue;
          int32_t hp = r->procs[i].hostpid.load(std::memory_order_relaxed);
          if (!hp) continue;
          int64_t v = kfd_cu_occupancy(hp, s.agents[d].gpu_id);
          if (v >= 0) {
            sum += v;
            any = true;
          }
        }
        if (any) {
          occ_sum[d] += sum;
          occ_ok[d]++;
        }
      }
      nanosleep(&tick, nullptr);
    }
    r->hdr.watcher_heartbeat.store(now_ns());
    for (int d = 0; d < s.n_agents; d++) {
      AgentInfo& a = s.agents[d];
      DeviceState& ds = r->dev[d];
      int util;
      if (occ_ok[d]) {
        int64_t avg = occ_sum[d] / occ_ok[d];
        util = a.cu_count ? (int)(avg * 100 / a.cu_count) : 0;
      } else {
        util = device_busy_percent(a.gpu_id);
        if (util < 0) util = 0;
      }
      if (util > 100) util = 100;
      ds.util_pct.store(util);
      if (a.temporal_active) {
        LimiterSpec spec{a.cu_count, a.max_waves_per_cu * 64};
        limiter_refill(ds, spec, ds.cu_limit_pct, util);
      }
      // Monitor-based usage (reference set_gpu_device_memory_monitor).
      uint64_t mon = 0;
      int32_t worst_pid = 0;
      int64_t worst = -1;
      for (int i = 0; i < kMaxProcs; i++) {
        if (!r->procs[i].pid.load(std::memory_order_relaxed)) continue;
        int32_t hp = r->procs[i].hostpid.load(std::memory_order_relaxed);
        if (!hp || !a.gpu_id) continue;
        int64_t v = kfd_vram_usage(hp, a.gpu_id);
        if (v > 0) {
          mon += (uint64_t)v;
          if (v > worst) {
            worst = v;
            worst_pid = r->procs[i].pid.load();
          }
        }
      }
      ds.monitor_used.store(mon);
      if ((r->hdr.flags & kFlagActiveOomKiller) && ds.mem_limit && mon > ds.mem_limit && worst_pid > 0) {
        VLOG_ERROR("device %d: measured usage %lu exceeds limit %lu; killing largest consumer pid %d", d,
                   (unsigned long)mon, (unsigned long)ds.mem_limit, worst_pid);
        kill(worst_pid, SIGKILL);
      }
    }
  }
  int32_t me32 = me;
  r->hdr.watcher_pid.compare_exchange_strong(me32, 0);
  return nullptr;
}

}  // namespace

void start_watcher_if_needed() {
  ShimState& s = shim();
  if (!s.active) return;
  const Config& cfg = config();
  bool need = cfg.active_oom_killer || cfg.memory_override;
  for (int i = 0; i < s.n_agents; i++) need |= s.agents[i].temporal_active;
  if (!need) return;
  bool expected = false;
  if (!s.watcher_started.compare_exchange_strong(expected, true)) return;
  pthread_t th;
  pthread_attr_t attr;
  pthread_attr_init(&attr);
  pthread_attr_setdetachstate(&attr, PTHREAD_CREATE_DETACHED);
  if (pthread_create(&th, &attr, watcher_main, nullptr) != 0) {
    VLOG_ERROR("cannot start utilisation watcher");
    s.watcher_started.store(false);
  }
  pthread_attr_destroy(&attr);
}

}  // namespace vgpu
