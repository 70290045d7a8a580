// Maintenance thread of every GPU process in a vGPU container, and the container's
// temporal-mode sampler.
//
// Reference: utilization_watcher@0x471a7 [multiprocess_utilization_watcher.c:195-216]
// retries the host-PID lookup while it is unknown, samples NVML per-process SM
// utilisation every 120 ms, sums it over the region's host PIDs, refills the token
// bucket through delta(), and feeds set_gpu_device_memory_monitor → active_oom_killer
// (SIGKILL every region process).
//
// MI355X: every process runs this thread for its own bookkeeping (host-PID discovery
// retries, continuous context accounting from KFD's vram counter, live limit changes).
// One process per region holds the sampler lease (watcher_pid + heartbeat) and does the
// container-wide work: in temporal mode it samples KFD cu_occupancy of the container's
// processes and of every other process on the GPU about every millisecond and turns it
// into the GPU-time credit of ratelimit.h; every period it updates monitor-based usage
// and runs the OOM killer, which terminates the largest consumer instead of every
// process.
#include <dirent.h>
#include <errno.h>
#include <pthread.h>
#include <signal.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <map>
#include <vector>

#include "shim.h"
#include "vgpu/board.h"
#include "vgpu/kfd.h"
#include "vgpu/ledger.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

namespace vgpu {

namespace {

// Device-wide busy percent for KFD gpu_id via the topology's render minor (fallback
// signal when none of the container's host PIDs is known yet).
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
  // EPERM means the holder exists (another user's process in the container): not stale.
  bool stale = cur == 0 || (kill(cur, 0) != 0 && errno == ESRCH) || (hb && now_ns() - hb > 1'000'000'000ull);
  if (!stale) return false;
  return r->hdr.watcher_pid.compare_exchange_strong(cur, me);
}

bool any_temporal() {
  ShimState& s = shim();
  for (int i = 0; i < s.n_agents; i++)
    if (s.agents[i].temporal_active.load(std::memory_order_relaxed)) return true;
  return false;
}

// Occupancy sampler state (lease holder only).
struct Sampler {
  uint64_t last_ns = 0;
  uint64_t others_at_ns = 0;
  std::vector<int> mine;                  // host PIDs of the container's processes
  int unknown = 0;                        // container processes whose host PID is unknown
  std::vector<int> others[kMaxDevices];   // other processes on each GPU
  int prev_pm[kMaxDevices] = {};          // charge fraction at the previous sample
  int64_t occ_ref[kMaxDevices] = {};      // decaying peak of the container's occupancy
  bool opened[kMaxDevices] = {};          // the previous sample re-opened the gate
  int procs = 1;                          // processes on the busiest sampled GPU (period)
  Board board;                            // node-wide board (VGPU_BOARD_DIR), if any
  bool board_tried = false;
  uint64_t yielded_ns[kMaxDevices] = {};  // background class: time spent yielding (diagnostics)
  uint64_t preempt_until[kMaxDevices] = {};  // background class: launches held until (strict yield)
  uint64_t want_since[kMaxDevices] = {};  // concurrency admission: waiting since (0 = not)
  uint64_t open_since[kMaxDevices] = {};  // concurrency admission: holding the GPU since
  bool admitted[kMaxDevices] = {};
  // Node ledger (vgpu/ledger.h): per device, the mapped file and this container's last
  // seen cumulative charge of each of its host PIDs.
  LedgerReader ledger[kMaxDevices];
  std::map<int, uint64_t> ledger_seen[kMaxDevices];
  uint64_t ledger_retry_ns[kMaxDevices] = {};
  uint64_t others_busy_ns[kMaxDevices] = {};  // last sample at which another process had waves resident
  uint64_t mem_refresh_ns = 0;                // next read of the peers' memory (memory_board_tick)
  uint64_t want_seen_ns[kMaxDevices] = {};    // the peers' HBM request already served
  // Automatic pair turns (VGPU_GPU_CONCURRENCY=auto): the container's launch rate and, per
  // GPU, whether its containers take turns in pairs now.
  uint64_t rate_launches = 0, rate_at_ns = 0;
  double launch_rate = 0;                     // kernel launches per second (EWMA)
  bool pairs_on[kMaxDevices] = {};
  uint64_t pairs_low_since[kMaxDevices] = {};
  // Steadiness (auto): of the samples at which the container was free to launch, the share
  // with launches or work of its own on the GPU since the previous one. A batch pod is busy at
  // every sample; a
  // request-serving pod idles between requests, and while one is busy on a GPU its pods do
  // not take pair turns: it would wait for them (profiles/r6a).
  uint64_t act_launches = 0;
  uint32_t act_ticks = 0, act_busy = 0;
  bool act_prev_free = false;
  double activity = 1.0;
  bool steady = true;
};

// A container launching fewer kernels per second than this is idle as far as the automatic
// pair turns are concerned, bursty or not.
constexpr uint32_t kBurstyMinRate = 500;

// The concurrency admission's k on device `d` (0 = everybody at once).
int concurrency_on(const Sampler& sm, int d) {
  const int k = sm.board.attached() ? config().gpu_concurrency : 0;
  return k >= 0 ? k : (sm.pairs_on[d] ? 2 : 0);
}

// The container's launches so far: this process's live counter, the others' as published.
uint64_t container_launches(const Region* r) {
  ShimState& s = shim();
  uint64_t total = s.launches.load(std::memory_order_relaxed);
  for (int i = 0; i < kMaxProcs; i++)
    if (i != s.slot && r->procs[i].pid.load(std::memory_order_relaxed))
      total += r->procs[i].launches.load(std::memory_order_relaxed);
  return total;
}

// VGPU_GPU_CONCURRENCY=auto (lease holder, every period): the container's launch rate from
// its processes' launch counters, published on the board; per GPU, pairs switch on while the
// GPU's containers together launch more than VGPU_PAIRS_ON_RATE kernels/s and off after
// kPairsOffNs below VGPU_PAIRS_OFF_RATE (the rates of a waiting container fall, those of the holders do not).
void pairs_tick(Region* r, Sampler& sm, const uint32_t* ids, uint64_t now) {
  ShimState& s = shim();
  uint64_t total = 0;
  for (int i = 0; i < kMaxProcs; i++)
    if (r->procs[i].pid.load(std::memory_order_relaxed)) total += r->procs[i].launches.load(std::memory_order_relaxed);
  if (sm.rate_at_ns && now > sm.rate_at_ns) {
    const double inst = total >= sm.rate_launches ? (double)(total - sm.rate_launches) * 1e9 / (now - sm.rate_at_ns) : 0;
    sm.launch_rate = 0.5 * sm.launch_rate + 0.5 * inst;
  }
  sm.rate_launches = total;
  sm.rate_at_ns = now;
  sm.board.publish_launch_rate((uint32_t)std::min(sm.launch_rate, 1e7));
  if (config().gpu_concurrency >= 0) return;
  if (sm.act_ticks >= 20) {
    sm.activity = 0.6 * sm.activity + 0.4 * ((double)sm.act_busy / sm.act_ticks);
    sm.act_ticks = sm.act_busy = 0;
    const bool steady = sm.steady ? sm.activity >= 0.6 : sm.activity >= 0.8;
    if (steady != sm.steady)
      VLOG_INFO("launching at %.0f %% of the samples: %s", sm.activity * 100,
                steady ? "steady" : "bursty, no pair turns on its GPU");
    sm.steady = steady;
  }
  sm.board.publish_steady(sm.steady);
  VLOG_DEBUG("container launch rate %.0f/s, %s", sm.launch_rate, sm.steady ? "steady" : "bursty");
  sm.board.refresh(now);
  for (int d = 0; d < s.n_agents; d++) {
    const uint64_t rate = (uint64_t)sm.launch_rate + sm.board.peers_launch_rate(ids[d]);
    // A busy bursty container on the GPU (a pod serving requests) would wait for turns: no
    // pairs there, whatever the rate (profiles/r6a).
    const bool bursty = (!sm.steady && sm.launch_rate >= kBurstyMinRate) || sm.board.bursty_peer_on(ids[d], kBurstyMinRate);
    if (bursty) {
      if (sm.pairs_on[d]) VLOG_INFO("device %d: a bursty container is busy on the GPU -> all at once", d);
      sm.pairs_on[d] = false;
      sm.pairs_low_since[d] = 0;
    } else if (rate >= config().pairs_on_rate) {
      if (!sm.pairs_on[d]) VLOG_INFO("device %d: %lu launches/s on the GPU -> pair turns", d, (unsigned long)rate);
      sm.pairs_on[d] = true;
      sm.pairs_low_since[d] = 0;
    } else if (sm.pairs_on[d] && rate < config().pairs_off_rate) {
      if (!sm.pairs_low_since[d]) sm.pairs_low_since[d] = now;
      if (now - sm.pairs_low_since[d] >= kPairsOffNs) {
        VLOG_INFO("device %d: %lu launches/s on the GPU -> all at once", d, (unsigned long)rate);
        sm.pairs_on[d] = false;
        sm.pairs_low_since[d] = 0;
      }
    } else {
      sm.pairs_low_since[d] = 0;
    }
  }
}

// The credit window of device `d`: the configured one, or the longer solo window while no
// other process has kept the GPU busy for a second. Alone on the GPU nobody waits behind
// the container's bursts, and every restart after an off period costs it warm-up (clocks,
// caches, an empty queue the host refills): four times fewer restarts recover most of a
// lone pod's loss under the GPU-time limiter (profiles/r3ae: 0.89 of its 25 % at 40 ms).
int window_ms(const Sampler& sm, int d, uint64_t now) {
  const Config& cfg = config();
  const bool solo = cfg.limiter_solo_window_ms > cfg.limiter_window_ms && now - sm.others_busy_ns[d] > 1'000'000'000ull;
  return solo ? cfg.limiter_solo_window_ms : cfg.limiter_window_ms;
}

// The node ledger of device `d` when the daemon keeps it fresh (re-mapped at most every
// 100 ms while absent), else null: the container then samples KFD by itself.
const LedgerReader* fresh_ledger(Sampler& sm, int d, uint32_t gpu_id, uint64_t now) {
  const Config& cfg = config();
  if (cfg.board_dir.empty() || !cfg.use_ledger || !gpu_id) return nullptr;
  LedgerReader& l = sm.ledger[d];
  if (l.attached() && l.fresh(now)) return &l;
  // Absent, or stale: a restarted daemon writes a new file under the same name, so a
  // stale mapping is dropped and the name opened again.
  if (now < sm.ledger_retry_ns[d]) return nullptr;
  sm.ledger_retry_ns[d] = now + 100'000'000ull;
  l.close();
  if (!l.open(cfg.board_dir, gpu_id) || !l.fresh(now)) return nullptr;
  sm.ledger_seen[d].clear();  // another file: cumulative charges start over
  return &l;
}

// Charge of the interval from the ledger: the growth of the cumulative charges of the
// container's processes since the last tick (a process seen for the first time starts
// from its current value).
int64_t ledger_charge(const LedgerReader& l, std::map<int, uint64_t>& seen, const std::vector<int>& mine,
                      int64_t* occ_out) {
  int64_t charge = 0, occ = 0;
  std::map<int, uint64_t> next;
  for (int hp : mine) {
    const LedgerEntry* e = l.find(hp);
    if (!e) continue;
    const uint64_t c = e->charged_ns.load(std::memory_order_relaxed);
    auto it = seen.find(hp);
    if (it != seen.end() && c >= it->second) charge += (int64_t)(c - it->second);
    next[hp] = c;
    occ += std::max(0, e->occ.load(std::memory_order_relaxed));
  }
  seen.swap(next);
  *occ_out = occ;
  return charge;
}

// The container's task priority (live: vgpuctl / the monitor may change it).
int region_priority(const Region* r) { return effective_priority(r); }

// Virtual device memory across containers (lease holder, every period): publishes the
// container's SVM bytes in each GPU's VRAM and any HBM it was refused within its quota; reads
// the peers' (every 250 ms while either matters here, else every second) into the region:
// the SVM VRAM of the other containers on each GPU (hidden_vram), and a demotion request when
// a peer on the GPU waits for HBM while this container holds promoted spills there - once per
// request (a peer re-publishes its request every second while it still waits).
void memory_board_tick(Region* r, Sampler& sm, const uint32_t* ids, uint64_t now) {
  ShimState& s = shim();
  bool mine = false;
  for (int d = 0; d < s.n_agents; d++) {
    DeviceState& ds = r->dev[d];
    const uint64_t svm = s.region.svm_vram(d);
    const uint64_t want_ns = ds.hbm_want_ns.load(std::memory_order_relaxed);
    const bool fresh = want_ns && now - want_ns < kBoardWantNs;
    sm.board.publish_memory(d, svm, fresh ? ds.hbm_want.load(std::memory_order_relaxed) : 0, want_ns);
    mine |= svm || fresh || ds.node_svm_vram.load(std::memory_order_relaxed);
  }
  if (now < sm.mem_refresh_ns) return;
  sm.mem_refresh_ns = now + (mine ? 250'000'000ull : 1'000'000'000ull);
  sm.board.refresh(now);
  for (int d = 0; d < s.n_agents; d++) {
    DeviceState& ds = r->dev[d];
    ds.node_svm_vram.store(sm.board.peers_svm_vram(ids[d]), std::memory_order_relaxed);
    uint64_t newest = 0;
    const uint64_t want = sm.board.peers_hbm_want(ids[d], &newest);
    const uint64_t svm = s.region.svm_vram(d);
    if (!want) {
      sm.want_seen_ns[d] = 0;
      ds.demote_want.store(0, std::memory_order_relaxed);
    } else if (newest != sm.want_seen_ns[d] && svm) {
      sm.want_seen_ns[d] = newest;
      ds.demote_want.store(std::min(want, svm), std::memory_order_relaxed);
      VLOG_INFO("device %d: a co-tenant waits for %lu bytes of HBM; demoting up to %lu bytes of promoted spills", d,
                (unsigned long)want, (unsigned long)std::min(want, svm));
    }
  }
}

// Publishes the container on the board (lease holder, every period).
void board_tick(Region* r, Sampler& sm, uint64_t now) {
  const Config& cfg = config();
  if (cfg.board_dir.empty()) return;
  if (!sm.board.attached()) {
    if (sm.board_tried) return;
    sm.board_tried = true;
    int rc = sm.board.open(cfg.board_dir.c_str(), cfg.board_slot.empty() ? "self.slot" : cfg.board_slot.c_str());
    if (rc != 0) {
      VLOG_WARN("cannot open board slot %s/%s (%s); priorities act without it", cfg.board_dir.c_str(),
                cfg.board_slot.c_str(), strerror(-rc));
      return;
    }
    shim().board_slot.store(sm.board.self());  // on_exit takes the container off the board
    sm.board.publish_cpu_node(cfg.cpu_node);
  }
  ShimState& s = shim();
  uint32_t ids[kMaxDevices];
  uint32_t masks[kMaxDevices][kCuMaskWords] = {};
  for (int i = 0; i < s.n_agents; i++) {
    ids[i] = s.agents[i].gpu_id;
    // A background tenant's own mask is derived from the reservation: not published, so
    // masks never feed back into each other.
    if (s.agents[i].mask_active.load(std::memory_order_relaxed) && region_priority(r) < kPrioBackground)
      memcpy(masks[i], s.agents[i].mask.words, sizeof(masks[i]));
  }
  sm.board.publish(region_priority(r), ids, s.n_agents, sm.mine, now, masks);
  memory_board_tick(r, sm, ids, now);
  pairs_tick(r, sm, ids, now);
  // Background class: keep off the CU slices of latency-class tenants on the same GPU.
  // Stored in the region, so every process of the container re-masks its queues.
  if (region_priority(r) < kPrioBackground) return;
  sm.board.refresh(now);
  bool changed = false;
  for (int i = 0; i < s.n_agents; i++) {
    uint32_t want[kCuMaskWords];
    sm.board.reserved_mask(ids[i], kPrioLatency, want);
    DeviceState& d = r->dev[i];
    if (memcmp(want, d.reserved_mask, sizeof(want)) != 0) {
      memcpy(d.reserved_mask, want, sizeof(want));
      changed = true;
    }
  }
  if (changed) r->hdr.generation.fetch_add(1, std::memory_order_acq_rel);
}

void collect_region_pids(Region* r, Sampler& sm) {
  sm.mine.clear();
  sm.unknown = 0;
  for (int i = 0; i < kMaxProcs; i++) {
    if (!r->procs[i].pid.load(std::memory_order_relaxed)) continue;
    int32_t hp = r->procs[i].hostpid.load(std::memory_order_relaxed);
    if (hp) sm.mine.push_back(hp);
    else sm.unknown++;
  }
}

// Background class, strict form (VGPU_PREEMPT_HOLD_MS / VGPU_PREEMPT_DEPTH). The soft
// yield only stops earning credit, so a background tenant keeps launching until its
// credit runs out while the better class waits behind its kernels on the memory system
// (profiles/r3k: the service's kernels run ~3x longer next to the trainers). Strict:
// (1) while a better class has waves resident, and for the hold time after, the gate is
// closed outright; (2) while a better-class tenant shares the GPU (board), each process
// keeps at most `depth` AQL packets in flight (gate_launch), so what is queued when the
// better class wakes up drains in a few kernels. HAMi-style preemption by priority, at
// launch granularity: running kernels are never interrupted.
void preempt_tick(Sampler& sm, DeviceState& ds, uint32_t gpu_id, int prio, int d, bool yield, uint64_t now) {
  const Config& cfg = config();
  if (cfg.preempt_hold_ms > 0) {
    if (yield) sm.preempt_until[d] = now + (uint64_t)cfg.preempt_hold_ms * 1'000'000ull;
    const bool held = now < sm.preempt_until[d];
    ds.preempt.store(held ? 1 : 0, std::memory_order_relaxed);
    if (held) ds.gate_open.store(0, std::memory_order_release);
  }
  const int cap = cfg.preempt_depth > 0 && sm.board.better_on(gpu_id, prio) ? cfg.preempt_depth : 0;
  if (ds.depth_cap.load(std::memory_order_relaxed) != cap) ds.depth_cap.store(cap, std::memory_order_relaxed);
}

void sample_tick(Region* r, Sampler& sm) {
  ShimState& s = shim();
  const uint64_t now = now_ns();
  const int64_t dt = sm.last_ns ? (int64_t)std::min<uint64_t>(now - sm.last_ns, 1'000'000'000ull) : 0;
  sm.last_ns = now;
  collect_region_pids(r, sm);
  const bool refresh = now - sm.others_at_ns > 100'000'000ull;
  bool any_conc = false;
  for (int d = 0; d < s.n_agents; d++) any_conc |= concurrency_on(sm, d) > 0;
  if (refresh) {
    sm.others_at_ns = now;
    sm.procs = 1;
  }
  // Peers: every sample for the concurrency admission, every 100 ms for the classes.
  if (any_conc || (refresh && sm.board.attached() && region_priority(r) >= kPrioBackground)) sm.board.refresh(now);
  for (int d = 0; d < s.n_agents; d++) {
    AgentInfo& a = s.agents[d];
    if (!a.temporal_active.load(std::memory_order_relaxed) || !a.gpu_id) {
      if (sm.admitted[d] || sm.want_since[d]) {  // left the limiter: give up the turn
        sm.admitted[d] = false;
        sm.want_since[d] = 0;
        sm.board.publish_gate(d, false, 0);
      }
      r->dev[d].preempt.store(0, std::memory_order_relaxed);  // and any strict-yield state
      r->dev[d].depth_cap.store(0, std::memory_order_relaxed);
      sm.preempt_until[d] = 0;
      // Off the limiter nothing is charged: the ledger's growth meanwhile must not be
      // charged on the way back either.
      sm.ledger_seen[d].clear();
      continue;
    }
    DeviceState& ds = r->dev[d];
    // (No host PID known yet: the device-wide fallback below, as without a ledger.)
    const LedgerReader* led = config().charge_model == ChargeModel::kShare && !(sm.mine.empty() && sm.unknown)
                                  ? fresh_ledger(sm, d, a.gpu_id, now)
                                  : nullptr;
    if (refresh) {
      std::vector<int> on = kfd_pids_on_gpu(a.gpu_id);
      sm.others[d].clear();
      for (int p : on)
        if (std::find(sm.mine.begin(), sm.mine.end(), p) == sm.mine.end()) sm.others[d].push_back(p);
      // The tick stretches with the processes on the GPU, ledger or not: with the ledger the
      // container reads nothing, but longer on/off periods of the gate are part of what
      // keeps a crowded GPU efficient (profiles/r2aj); the ledger's charge is integrated at
      // its own period whatever the tick.
      sm.procs = std::max(sm.procs, (int)(sm.mine.size() + sm.others[d].size()));
    }
    int pm = 0;  // the container's share of the GPU at this instant, per mille
    // Background class: no credit is earned while a higher-priority tenant (by its board
    // slot; a process on no slot counts as normal) has waves resident on this GPU.
    const int prio = region_priority(r);
    const bool background = prio >= kPrioBackground;
    bool yield = false;
    int64_t led_charge = -1;
    if (led) {
      // The node ledger holds every process's charge from one snapshot per period: no
      // occupancy reads here at all.
      int64_t mine = 0;
      // At most the interval's wall time (the processes' shares of one snapshot add up to
      // at most 1), plus one ledger period of misalignment between the two clocks.
      led_charge = std::min<int64_t>(ledger_charge(*led, sm.ledger_seen[d], sm.mine, &mine),
                                     dt + (int64_t)led->file()->period_ns.load(std::memory_order_relaxed));
      const int64_t total = std::max<int64_t>(mine, led->file()->total_occ.load(std::memory_order_relaxed));
      if (total > mine) sm.others_busy_ns[d] = now;
      pm = (int)timeshare_charge(1000, mine, total);
      if (background)
        for (int p : sm.others[d]) {
          const LedgerEntry* e = led->find(p);
          if (e && e->occ.load(std::memory_order_relaxed) > 0 && sm.board.priority_of(p, a.gpu_id) < prio) {
            yield = true;
            break;
          }
        }
    } else if (!sm.mine.empty() || background) {
      int64_t mine = 0;
      for (int hp : sm.mine) mine += std::max<int64_t>(0, kfd_cu_occupancy(hp, a.gpu_id));
      // Split the instant with whoever else has waves resident on this GPU (other
      // containers, unlimited processes): only read when the container is busy (or
      // yields by class, which needs to know whether its betters are busy).
      int64_t total = mine;
      if (mine > 0 || background) {
        for (int p : sm.others[d]) {
          const int64_t occ = std::max<int64_t>(0, kfd_cu_occupancy(p, a.gpu_id));
          if (occ > 0) sm.others_busy_ns[d] = now;
          total += occ;
          if (background && occ > 0 && !yield && sm.board.priority_of(p, a.gpu_id) < prio) yield = true;
        }
        r->hdr.other_refreshes.fetch_add(1, std::memory_order_relaxed);
      }
      pm = (int)timeshare_charge(1000, mine, total);
      sm.occ_ref[d] = occupancy_ref_update(sm.occ_ref[d], mine);
      if (config().charge_model == ChargeModel::kProgress) pm = timeshare_progress_pm(pm, mine, sm.occ_ref[d]);
    } else if (sm.unknown) {
      // No host PID known yet: fall back to device-wide busy time (conservative).
      int busy = device_busy_percent(a.gpu_id);
      pm = busy > 0 ? std::min(busy, 100) * 10 : 0;
    }
    const int64_t charge = led_charge >= 0 ? led_charge : timeshare_interval(dt, sm.prev_pm[d], pm, sm.opened[d]);
    const bool was_closed = !ds.gate_open.load(std::memory_order_relaxed);
    if (yield) sm.yielded_ns[d] += dt;
    // The exact share (e.g. 6.25 % for split 16) only with the ledger's exact charges: the
    // container's own sampling over-charges on a crowded GPU (its charges add up to ~107 %
    // of the wall time at 16 pods), so it keeps the rounded-up whole percent, which leaves
    // room for that (the plugin emits the percent rounded up for this reason).
    timeshare_apply(ds, timeshare_params(ds.cu_limit_pct, window_ms(sm, d, now), led ? ds.cu_share_bp : 0), dt,
                    charge, yield ? 0 : dt);
    if (d == 0 && config().gpu_concurrency < 0) {
      // Steadiness: only samples at which the container was free to launch count.
      const uint64_t total = container_launches(r);
      // Free for the whole interval: not waiting for a turn, and the credit gate open at this
      // sample and the previous one (a pod the limiter throttles is not idle by choice).
      const bool free_now = !sm.want_since[d] && ds.gate_open.load(std::memory_order_relaxed);
      if (free_now && sm.act_prev_free) {
        sm.act_ticks++;
        // Busy: it launched, or work of its own was queued or resident meanwhile (a batch pod
        // waiting for its kernels is not idle; a serving pod between requests has nothing
        // on the GPU).
        if (total != sm.act_launches || charge > 0 || packets_queued(d) > 0) sm.act_busy++;
      }
      sm.act_prev_free = free_now;
      sm.act_launches = total;
    }
    const int conc = concurrency_on(sm, d);
    if (conc <= 0 && (sm.admitted[d] || sm.want_since[d])) {  // pairs switched off: out of the turns
      sm.admitted[d] = false;
      sm.want_since[d] = 0;
      sm.board.publish_gate(d, false, 0);
    }
    if (conc > 0) {
      // Concurrency admission, round robin: while its credit allows, a container holds
      // the GPU for a slice, then yields to the longest-waiting peer; at most `conc`
      // containers of the GPU hold it at once. The containers take turns in small groups
      // instead of all overlapping (the credit still caps each one's share). Three or more
      // processes with launches in flight on one GPU each dispatch at a quarter of the rate
      // two reach (profiles/r6f: a CP-side cross-process cost, not the CPU), and two on one
      // CPU socket run no faster than one (profiles/r5d): with CPU nodes known the groups
      // are cross-socket (Board::admit).
      const bool credit_ok = ds.gate_open.load(std::memory_order_relaxed);
      const int64_t slice = (int64_t)config().gpu_slice_ms * 1'000'000ll;
      bool hold = false;
      if (!credit_ok) {
        if (sm.admitted[d] || sm.want_since[d]) VLOG_DEBUG("device %d: no credit, out of the turns", d);
        sm.admitted[d] = false;
        sm.want_since[d] = 0;
      } else if (sm.admitted[d]) {
        hold = true;
        if ((int64_t)(now - sm.open_since[d]) >= slice && sm.board.waiting(a.gpu_id, conc, config().cpu_node)) {
          sm.admitted[d] = false;  // slice used up and someone waits: to the back of the queue
          sm.want_since[d] = now;
          hold = false;
          g_turn_held_ns.fetch_add(now - sm.open_since[d], std::memory_order_relaxed);
          VLOG_DEBUG("device %d: turn over after %.1f ms (CPU node %d)", d, (now - sm.open_since[d]) / 1e6,
                     config().cpu_node);
        }
      } else {
        if (!sm.want_since[d]) sm.want_since[d] = now;
        if (sm.board.admit(a.gpu_id, conc, sm.want_since[d], config().cpu_node)) {
          VLOG_DEBUG("device %d: admitted after %.1f ms of waiting (CPU node %d)", d,
                     (now - sm.want_since[d]) / 1e6, config().cpu_node);
          const uint64_t waited = now - sm.want_since[d];
          g_turns.fetch_add(1, std::memory_order_relaxed);
          g_turn_wait_ns.fetch_add(waited, std::memory_order_relaxed);
          if (waited > g_turn_wait_max_ns.load(std::memory_order_relaxed))
            g_turn_wait_max_ns.store(waited, std::memory_order_relaxed);
          sm.admitted[d] = true;
          sm.open_since[d] = now;
          sm.want_since[d] = 0;
          hold = true;
        }
      }
      if (!hold) ds.gate_open.store(0, std::memory_order_release);
      sm.board.publish_gate(d, hold, sm.want_since[d]);
    }
    if (background) {
      preempt_tick(sm, ds, a.gpu_id, prio, d, yield, now);
    } else {
      // On the limiter of a crowded GPU (three or more processes on it), a bounded queue
      // (VGPU_CROWD_DEPTH) keeps each pod's debt to a few kernels: the credit gate then paces
      // it kernel by kernel instead of admitting a whole synchronize-to-synchronize batch at
      // once (profiles/r5c). A pod alone under a GPU-time limit keeps its full queue. Counted
      // on this GPU: a crowded GPU of a multi-GPU container does not bound the others.
      const int on_gpu = (int)(sm.mine.size() + sm.others[d].size());
      const int cap = on_gpu > 2 ? config().crowd_depth : 0;
      if (ds.depth_cap.load(std::memory_order_relaxed) != cap) ds.depth_cap.store(cap, std::memory_order_relaxed);
    }
    sm.opened[d] = was_closed && ds.gate_open.load(std::memory_order_relaxed);
    sm.prev_pm[d] = pm;
  }
  r->hdr.samples.fetch_add(1, std::memory_order_relaxed);
  r->hdr.watcher_heartbeat.store(now);
}

// Auto mode below a 50 % share (lease holder, every period): how many other processes
// keep each GPU busy. A process counts while it had waves resident in the last 5 s (long
// enough to bridge the CPU-bound phases of a busy tenant, e.g. kernel compilation).
// One or none: the container keeps its CU mask (no duty-cycling, its own CUs); more: the
// masks of several tenants would stall each other in the dispatchers, so every
// container switches to the GPU-time limiter at once, and back after 2 s of calm.
struct Crowd {
  std::map<int, uint64_t> busy_at[kMaxDevices];  // other host PID -> last time with waves
  uint64_t calm_since[kMaxDevices] = {};
};

void crowd_tick(Region* r, Sampler& sm, Crowd& c, uint64_t now) {
  ShimState& s = shim();
  const Config& cfg = config();
  if (cfg.cu_mode != CuMode::kAuto) return;
  bool changed = false;
  for (int d = 0; d < s.n_agents; d++) {
    AgentInfo& a = s.agents[d];
    DeviceState& ds = r->dev[d];
    const int pct = ds.cu_limit_pct;
    // Assessed for every limited device (not only below 50 %), so a live change to a
    // smaller share finds the crowd already known; and for every device of a background
    // tenant, which goes on the GPU-time gate as soon as anyone else is busy.
    const bool background = region_priority(r) >= kPrioBackground;
    if (!a.gpu_id || ((pct <= 0 || pct >= 100) && !background)) continue;
    // From the node ledger when it is fresh: busy means waves resident at any of its
    // samples since the last tick, not only at this instant.
    const LedgerReader* led = fresh_ledger(sm, d, a.gpu_id, now);
    for (int p : kfd_pids_on_gpu(a.gpu_id)) {
      if (std::find(sm.mine.begin(), sm.mine.end(), p) != sm.mine.end()) continue;
      if (led) {
        const LedgerEntry* e = led->find(p);
        const uint64_t b = e ? e->busy_ns.load(std::memory_order_relaxed) : 0;
        if (b && (b > now || now - b < 150'000'000ull)) c.busy_at[d][p] = std::min(b, now);
        continue;
      }
      if (kfd_cu_occupancy(p, a.gpu_id) > 0) c.busy_at[d][p] = now;
    }
    int busy = 0;
    for (auto it = c.busy_at[d].begin(); it != c.busy_at[d].end();) {
      if (now - it->second > 5'000'000'000ull) {
        it = c.busy_at[d].erase(it);
      } else {
        busy++;
        ++it;
      }
    }
    const int cur = ds.crowd.load(std::memory_order_relaxed);
    // The count at which the enforcement changes: a background tenant switches to the
    // GPU-time gate as soon as one other process is busy (effective_cu_mode_prio).
    const int threshold = background ? 0 : kAutoSpatialMaxCrowd;
    const bool crowded_now = busy > threshold;
    const bool was_crowded = cur < 0 || cur > threshold;
    int next = busy;
    if (crowded_now || cur < 0) {
      c.calm_since[d] = 0;
    } else if (was_crowded) {  // calming down: hold the limiter for 2 s first
      if (!c.calm_since[d]) c.calm_since[d] = now;
      if (now - c.calm_since[d] < 2'000'000'000ull) next = cur;
    }
    if (next != cur) {
      ds.crowd.store(next, std::memory_order_relaxed);
      if ((next > threshold) != was_crowded) {
        changed = true;
        VLOG_INFO("device %d: %d other busy process(es) on the GPU -> %s", d, busy,
                  next > threshold ? "GPU-time limiter" : "CU mask");
      }
    }
  }
  if (changed) r->hdr.generation.fetch_add(1, std::memory_order_acq_rel);  // every process re-applies
}

// Monitor-based usage (reference set_gpu_device_memory_monitor) and the active OOM killer.
// The killer is the backstop for memory no hook saw (raw KFD ioctls, a runtime loaded
// around the shim, runtime-internal growth - scratch, queues - that is charged without
// admission): it acts when KFD's measured VRAM of the container stays above its quota plus
// a slack (max(512 MiB, 1/16 of the quota): the context charge may legitimately overshoot
// a little) for two consecutive periods. On by default as in the reference
// (ACTIVE_OOM_KILLER unset = on); under a plugin limits file the tenant cannot turn it off.
constexpr uint64_t kOomSlackMin = 512ull << 20;
void monitor_tick(Region* r) {
  ShimState& s = shim();
  static int over_ticks[kMaxDevices];
  const bool killer = config().active_oom_killer || (r->hdr.flags & kFlagActiveOomKiller);
  for (int d = 0; d < s.n_agents; d++) {
    AgentInfo& a = s.agents[d];
    DeviceState& ds = r->dev[d];
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
    const uint64_t limit = s.region.limit(d);  // the region's, within this process's ceiling
    const uint64_t slack = std::max<uint64_t>(kOomSlackMin, limit / 16);
    if (!killer || !limit || mon <= limit + slack || worst_pid <= 0) {
      over_ticks[d] = 0;
      continue;
    }
    if (++over_ticks[d] < 2) continue;
    over_ticks[d] = 0;
    VLOG_ERROR("device %d: measured usage %lu exceeds limit %lu (+%lu slack); killing largest consumer pid %d", d,
               (unsigned long)mon, (unsigned long)limit, (unsigned long)slack, worst_pid);
    for (int i = 0; i < kMaxProcs; i++)
      if (r->procs[i].pid.load(std::memory_order_relaxed) == worst_pid) r->procs[i].oom_events.fetch_add(1);
    kill(worst_pid, SIGKILL);
  }
}

void* watcher_main(void*) {
  ShimState& s = shim();
  Region* r = s.region.raw();
  const Config& cfg = config();
  const pid_t me = getpid();
  const uint64_t period_ns = (uint64_t)cfg.util_period_ms * 1'000'000ull;
  Sampler sm;
  Crowd crowd;
  uint64_t next_slow = 0, next_touch = 0;
  int pid_attempts = 0;
  unsigned rng = (unsigned)me * 2654435761u;
  while (!s.exiting.load() && s.pid == me) {
    const uint64_t now = now_ns();
    const bool lease = take_lease(r, me);
    const bool temporal = any_temporal();
    if (lease && temporal) {
      sample_tick(r, sm);
    } else {
      sm.last_ns = 0;
      for (auto& seen : sm.ledger_seen) seen.clear();  // nothing charged meanwhile (sample_tick)
    }
    if (now >= next_slow) {
      next_slow = now + period_ns;
      check_live_config();
      // Host-PID retries: every period for the first ~10 s, then every ~5 s.
      if (!s.hostpid && (pid_attempts < 80 || pid_attempts % 40 == 0)) {
        pid_t hp = resolve_hostpid(50);
        if (hp && s.slot >= 0) {
          s.hostpid = hp;
          r->procs[s.slot].hostpid.store(hp);
          VLOG_INFO("host PID %d resolved by the maintenance thread after %d attempt(s)", (int)hp, pid_attempts + 1);
        }
      }
      if (!s.hostpid) pid_attempts++;
      check_region_epoch();
      if (now >= next_touch) {  // a live container's region file keeps a fresh mtime (contract.py GC)
        next_touch = now + 10'000'000'000ull;
        s.region.touch();
      }
      if (s.slot >= 0) r->procs[s.slot].launches.store(s.launches.load(std::memory_order_relaxed));
      resync_context_charge();
      svm_tenant_reconcile();  // the tenant's SVM ranges it unmapped give their charge back
      publish_svm_vram();      // for the node board (hidden_vram)
      if (lease) {
        collect_region_pids(r, sm);
        board_tick(r, sm, now);
        crowd_tick(r, sm, crowd, now);
        monitor_tick(r);
        if (!temporal) r->hdr.watcher_heartbeat.store(now_ns());
      }
    }
    // Sampling cadence with ±25 % jitter so the samples never phase-lock to the gate,
    // stretched on a crowded GPU so the node's occupancy reads stay bounded.
    int64_t sleep_ns;
    if (lease && temporal) {
      rng = rng * 1103515245u + 12345u;
      int64_t base = sample_period_ns((int64_t)cfg.util_sample_us * 1000, (int64_t)sm.procs * sm.procs,
                                      cfg.sample_read_budget,
                                      std::max<int64_t>(10'000'000, (int64_t)cfg.util_sample_us * 1000));
      sleep_ns = base * 3 / 4 + (int64_t)((rng >> 8) % (uint32_t)(base / 2 + 1));
    } else {
      sleep_ns = (int64_t)std::min<uint64_t>(period_ns, next_slow > now_ns() ? next_slow - now_ns() : 0);
      if (sleep_ns < 1'000'000) sleep_ns = 1'000'000;
    }
    struct timespec ts = {(time_t)(sleep_ns / 1000000000), (long)(sleep_ns % 1000000000)};
    nanosleep(&ts, nullptr);
  }
  int32_t me32 = me;
  r->hdr.watcher_pid.compare_exchange_strong(me32, 0);
  return nullptr;
}

}  // namespace

void start_watcher_if_needed() {
  ShimState& s = shim();
  if (!s.active) return;
  // Always: the thread also publishes the launch counter and applies live limit changes
  // (it sleeps a whole period, 120 ms, between ticks unless the sampler runs).
  bool expected = false;
  if (!s.watcher_started.compare_exchange_strong(expected, true)) return;
  pthread_t th;
  pthread_attr_t attr;
  pthread_attr_init(&attr);
  pthread_attr_setdetachstate(&attr, PTHREAD_CREATE_DETACHED);
  if (pthread_create(&th, &attr, watcher_main, nullptr) != 0) {
    VLOG_ERROR("cannot start the maintenance thread");
    s.watcher_started.store(false);
  }
  pthread_attr_destroy(&attr);
}

}  // namespace vgpu
