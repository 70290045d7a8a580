// Shim lifecycle: lazy init inside hsa_init, fork/exit handling, launch gates.
#include "shim.h"

#include <pthread.h>
#include <signal.h>
#include <strings.h>
#include <sys/auxv.h>
#include <sys/stat.h>

#include <cerrno>
#include <new>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <ctime>
#include <string>
#include <vector>

#include "real.h"
#include "vgpu/board.h"
#include "vgpu/devmap.h"
#include "vgpu/kfd.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

namespace vgpu {

bool g_stats_on = false;
std::atomic<uint64_t> g_stats[kStatCount];
std::atomic<uint64_t> g_turns{0}, g_turn_held_ns{0}, g_turn_wait_ns{0}, g_turn_wait_max_ns{0};

namespace {
const char* const kStatNames[kStatCount] = {"hsa_agent_get_info", "hsa_amd_memory_pool_get_info",
                                            "hsa_amd_memory_pool_allocate", "hsa_amd_memory_pool_free",
                                            "hsa_queue_create", "hsa_amd_queue_cu_set_mask", "kernel launches",
                                            "hipGraphLaunch", "memcpy", "memset"};

void print_stats() {
  fprintf(stderr, "[vGPU stats pid %d]", (int)getpid());
  if (g_turns.load())
    fprintf(stderr, " turns=%lu held_ms=%.1f waited_ms=%.1f max_wait_ms=%.1f", (unsigned long)g_turns.load(),
            g_turn_held_ns.load() / 1e6, g_turn_wait_ns.load() / 1e6, g_turn_wait_max_ns.load() / 1e6);
  for (int i = 0; i < kStatCount; i++) fprintf(stderr, " %s=%lu", kStatNames[i], (unsigned long)g_stats[i].load());
  fprintf(stderr, " blocking_waits=%lu polled=%lu wait_ms=%.1f wakeups=%lu active_waits=%lu active_ms=%.1f\n",
          (unsigned long)g_sync_waits.load(), (unsigned long)g_sync_polled.load(), g_sync_wait_ns.load() / 1e6,
          (unsigned long)g_sync_wakeups.load(), (unsigned long)g_sync_active.load(), g_sync_active_ns.load() / 1e6);
}

__attribute__((constructor)) void stats_ctor() {
  const char* s = getenv("VGPU_STATS");
  if (s && *s && *s != '0') {
    g_stats_on = true;
    atexit(print_stats);
  }
}
}  // namespace

ShimState& shim() {
  static ShimState* s = new ShimState();  // never destroyed: hooks may run during exit
  return *s;
}

namespace {

struct AgentScan {
  ShimState* s;
  hsa_agent_t cpus[kMaxDevices];
  int n_cpu;
};

hsa_status_t pool_cb(hsa_amd_memory_pool_t pool, void* data) {
  AgentInfo* a = static_cast<AgentInfo*>(data);
  VGPU_REAL_HSA(hsa_amd_memory_pool_get_info);
  hsa_amd_segment_t seg;
  if (real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS)
    return HSA_STATUS_SUCCESS;
  if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
  if (a->n_pools < kMaxAgentPools) a->pools[a->n_pools++] = pool;
  size_t sz = 0;
  uint32_t flags = 0;
  real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &sz);
  real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  if ((flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED) && sz > a->phys_total) {
    a->phys_total = sz;
    bool alloc_ok = false;
    real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc_ok);
    if (alloc_ok) a->vram_pool = pool;
  }
  return HSA_STATUS_SUCCESS;
}

// The agent's global regions (legacy hsa_memory_allocate API): in ROCr a region handle and
// the pool handle of the same memory are one object, but that is not part of the API, so
// the handles are recorded with the pools either way (pool_ordinal covers both).
hsa_status_t region_cb(hsa_region_t region, void* data) {
  AgentInfo* a = static_cast<AgentInfo*>(data);
  VGPU_REAL_HSA(hsa_region_get_info);
  hsa_region_segment_t seg;
  if (!real_hsa_region_get_info ||
      real_hsa_region_get_info(region, HSA_REGION_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_REGION_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  for (int j = 0; j < a->n_pools; j++)
    if (a->pools[j].handle == region.handle) return HSA_STATUS_SUCCESS;
  if (a->n_pools < kMaxAgentPools) a->pools[a->n_pools++] = hsa_amd_memory_pool_t{region.handle};
  return HSA_STATUS_SUCCESS;
}

// Every global pool of a CPU agent: allocations from them pin host memory (host_hooks.cpp).
hsa_status_t cpu_pool_record_cb(hsa_amd_memory_pool_t pool, void* data) {
  ShimState* s = static_cast<ShimState*>(data);
  VGPU_REAL_HSA(hsa_amd_memory_pool_get_info);
  hsa_amd_segment_t seg;
  if (real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  for (int i = 0; i < s->n_cpu_pools; i++)
    if (s->cpu_pools[i].handle == pool.handle) return HSA_STATUS_SUCCESS;
  if (s->n_cpu_pools < kMaxAgentPools) s->cpu_pools[s->n_cpu_pools++] = pool;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t cpu_pool_cb(hsa_amd_memory_pool_t pool, void* data) {
  AgentInfo* a = static_cast<AgentInfo*>(data);
  VGPU_REAL_HSA(hsa_amd_memory_pool_get_info);
  hsa_amd_segment_t seg;
  uint32_t flags = 0;
  bool alloc_ok = false;
  if (real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg) != HSA_STATUS_SUCCESS ||
      seg != HSA_AMD_SEGMENT_GLOBAL)
    return HSA_STATUS_SUCCESS;
  real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
  real_hsa_amd_memory_pool_get_info(pool, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc_ok);
  if (!alloc_ok || (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT)) return HSA_STATUS_SUCCESS;
  // Prefer coarse-grained host memory for spill (no coherence traffic); a fine
  // grained pool is the fallback.
  if (!a->spill_pool.handle || (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) a->spill_pool = pool;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t agent_cb(hsa_agent_t agent, void* data) {
  AgentScan* sc = static_cast<AgentScan*>(data);
  VGPU_REAL_HSA(hsa_agent_get_info);
  hsa_device_type_t type;
  if (real_hsa_agent_get_info(agent, HSA_AGENT_INFO_DEVICE, &type) != HSA_STATUS_SUCCESS) return HSA_STATUS_SUCCESS;
  if (type == HSA_DEVICE_TYPE_CPU) {
    if (sc->n_cpu < kMaxDevices) sc->cpus[sc->n_cpu++] = agent;
    return HSA_STATUS_SUCCESS;
  }
  if (type != HSA_DEVICE_TYPE_GPU || sc->s->n_agents >= kMaxDevices) return HSA_STATUS_SUCCESS;
  AgentInfo& a = sc->s->agents[sc->s->n_agents++];
  a.agent = agent;
  uint32_t v = 0;
  if (real_hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT, &v) == HSA_STATUS_SUCCESS)
    a.cu_count = (int)v;
  v = 1;
  if (real_hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NUM_XCC, &v) == HSA_STATUS_SUCCESS && v)
    a.num_xcc = (int)v;
  v = 0;
  if (real_hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NUM_SHADER_ENGINES, &v) == HSA_STATUS_SUCCESS &&
      v) {
    // Reported for the whole agent on multi-XCC parts; normalise to per XCC.
    a.num_se = (v >= (uint32_t)a.num_xcc && v % a.num_xcc == 0) ? (int)(v / a.num_xcc) : (int)v;
  }
  v = 0;
  if (real_hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DRIVER_UID, &v) == HSA_STATUS_SUCCESS)
    a.gpu_id = v;
  v = 0;
  if (real_hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MAX_WAVES_PER_CU, &v) == HSA_STATUS_SUCCESS && v)
    a.max_waves_per_cu = (int)v;
  hsa_agent_t cpu{0};
  if (real_hsa_agent_get_info(agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_NEAREST_CPU, &cpu) == HSA_STATUS_SUCCESS)
    a.cpu_agent = cpu;
  VGPU_REAL_HSA(hsa_amd_agent_iterate_memory_pools);
  real_hsa_amd_agent_iterate_memory_pools(agent, pool_cb, &a);
  VGPU_REAL_HSA(hsa_agent_iterate_regions);
  if (real_hsa_agent_iterate_regions) real_hsa_agent_iterate_regions(agent, region_cb, &a);
  return HSA_STATUS_SUCCESS;
}

void on_signal_suspend(int) {
  ShimState& s = shim();
  if (s.slot >= 0 && s.region.attached()) s.region.raw()->procs[s.slot].status.store(kProcSuspended);
}
void on_signal_resume(int) {
  ShimState& s = shim();
  if (s.slot >= 0 && s.region.attached()) s.region.raw()->procs[s.slot].status.store(kProcRunning);
}

// fork() while another thread is inside an allocation hook: the allocation table must
// not be copied half-updated, and the child (which has only the forking thread) must not
// inherit a lock that thread can never release. The table's lock is taken around the
// fork; in the child both locks are re-created unlocked.
void atfork_prepare() {
  shim().alloc_mu.lock();
  shim().queue_mu.lock();
}
void atfork_parent() {
  shim().queue_mu.unlock();
  shim().alloc_mu.unlock();
}

void atfork_child() {
  // A forked child is a different process: it must not inherit the parent's slot
  // or allocation records (reference: child_reinit_flag). ROCr state does not
  // survive fork either, so the child re-initialises if it calls hsa_init again.
  ShimState& s = shim();
  new (&s.alloc_mu) std::mutex();  // held by this thread since atfork_prepare
  new (&s.live_mu) std::mutex();   // may be held by a parent thread that does not exist here
  new (&s.ctx_mu) std::mutex();
  new (&s.queue_mu) std::mutex();  // held by this thread since atfork_prepare
  s.slot = -1;
  s.active = false;
  s.allocs.clear();
  s.vmem.clear();
  s.managed.clear();
  s.ipc.clear();
  s.host.clear();
  s.vcharge.clear();
  svm_forget();
  svm_tenant_forget();
  for (auto& b : s.ipc_bytes) b.store(0);
  s.queues.clear();
  s.hostpid = 0;
  s.launches.store(0);
  s.watcher_started.store(false);
  s.board_slot.store(nullptr);
  s.phase.store(0);
  s.pid = getpid();
}

void on_exit() {
  ShimState& s = shim();
  s.exiting.store(true);
  // The lease holder leaves the board at once: peers waiting for admission must not count
  // its gates as open until its heartbeat goes stale. Another process of the container
  // takes the lease and publishes again.
  if (BoardSlot* b = static_cast<BoardSlot*>(s.board_slot.load())) {
    for (auto& g : b->gate) g.store(0, std::memory_order_relaxed);
    b->heartbeat_ns.store(0, std::memory_order_release);
  }
  if (s.slot >= 0 && s.region.attached() && s.pid == getpid()) {
    s.region.raw()->procs[s.slot].launches.store(s.launches.load());
    // Reference exit_handler [475-494]: release the slot and its charges.
    s.region.unregister_process(s.slot);
    s.slot = -1;
  }
}

void load_env_config() {
  // Secure-execution mode (setuid/setgid or file capabilities): /etc/ld.so.preload still
  // loads the shim, but the environment belongs to the less privileged caller, so none
  // of it (region path, override file, limits) may steer a privileged process. The shim
  // stays a pass-through there.
  if (getauxval(AT_SECURE)) {
    mutable_config().disabled = true;
    return;
  }
  log_init_from_env();
  // Alternate KFD process tree (the CPU-only fake runtime of the test suite). Not in a real
  // container (the plugin's limits file mounted): a tenant's fake occupancy / VRAM files
  // would steer its own charges.
  if (const char* k = getenv("VGPU_KFD_ROOT"))
    if (*k && access(kLimitsPath, F_OK) != 0) g_kfd_proc_root = strdup(k);
  const char* ovr = getenv("VGPU_OVERRIDE_ENV_FILE");
  int n = apply_override_env_file(ovr && *ovr ? ovr : "/vgpu/override.env");
  if (n) log_init_from_env();
  Config& cfg = mutable_config();
  load_config(&cfg);
  if (n) VLOG_INFO("applied %d override env entries", n);
  // The plugin's ceilings: its read-only limits file at the fixed container path and, for
  // runs without a container runtime (tests, the bench's emulated pods), the one named by
  // VGPU_LIMITS_FILE. Each only lowers what the environment asks for.
  const char* extra = getenv("VGPU_LIMITS_FILE");
  const char* paths[2] = {kLimitsPath, extra && *extra && strcmp(extra, kLimitsPath) != 0 ? extra : nullptr};
  for (const char* p : paths) {
    if (!p) continue;
    Config ceil;
    if (!load_ceiling(p, &ceil)) {
      if (p == extra) VLOG_WARN("VGPU_LIMITS_FILE=%s is not readable", p);
      continue;
    }
    apply_ceiling(&cfg, ceil);
    shim().has_ceiling = true;
    VLOG_INFO("limits file %s applied (priority class floor %d)", p, ceil.min_priority);
  }
}

// Resolves the plugin's per-vGPU ceilings onto the agents (same map as the config) and
// installs them in the region handle and the agents.
void install_ceilings(const char* const* uuid_ptrs) {
  ShimState& s = shim();
  if (!s.has_ceiling) return;
  // The ceiling equals the clamped config: apply_ceiling took the map, and every per-device
  // limit is at most the file's; the file's own values are re-read for the mask.
  const char* extra = getenv("VGPU_LIMITS_FILE");
  Config ceil;
  if (!load_ceiling(kLimitsPath, &ceil) && !(extra && *extra && load_ceiling(extra, &ceil))) return;
  if (extra && *extra && strcmp(extra, kLimitsPath) != 0 && ceil.ceiling) {
    Config second;
    if (load_ceiling(extra, &second)) apply_ceiling(&ceil, second);
  }
  DeviceMap map;
  if (!parse_device_map(config().device_map.c_str(), &map)) map = DeviceMap();
  DeviceConfig per[kMaxDevices];
  resolve_devices(ceil, map, uuid_ptrs, s.n_agents, per);
  s.region.set_host_ceiling(ceil.host_mem_limit);
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    // A device the map does not give this container gets nothing (it is unauthorised too).
    s.region.set_ceiling(i, per[i].unmapped ? 1 : per[i].mem_limit);
    s.region.set_hbm_ceiling(i, per[i].hbm_limit);
    const int pct = per[i].cu_limit_pct;
    if (pct > 0 && pct < 100) {
      a.ceil_pct = pct;
      // The grant basis: the file's exact share, or its whole-percent limit.
      a.ceil_share_bp = per[i].cu_share_bp > 0 ? per[i].cu_share_bp : pct * 100;
      const char* layout = getenv("VGPU_CU_LAYOUT");
      a.ceil_mask = cu_mask_for(a.cu_count, a.num_xcc, pct, per[i].cu_range_begin, per[i].cu_range_end,
                                (layout && !strcasecmp(layout, "interleave")) ? 1 : a.num_se);
    }
  }
}

// Fills the region's per-device state from the resolved config where no process of the
// container has yet (d.configured == 0). Called with the region lock held. The resolved
// limits win over what is there: a region first created by a process that never
// initialised ROCr (amd-smi, torch's device count through amdsmi) holds the raw
// per-vGPU values of the environment, not the per-agent ones - for two vGPUs of one GPU,
// vGPU 0's quota where the merged GPU has both.
void configure_devices(Region* r, const DeviceConfig* per_agent, const Config& resolved) {
  ShimState& s = shim();
  if (r->hdr.num_devices < s.n_agents) r->hdr.num_devices = s.n_agents;
  // Split duplicate vGPUs: their own quota slots after the agents' (vdev_hooks.cpp).
  for (int i = s.n_agents; i < resolved.num_devices && i < kMaxDevices; i++) {
    DeviceState& d = r->dev[i];
    if (d.configured) continue;
    snprintf(d.uuid, sizeof(d.uuid), "%.63s", resolved.dev[i].uuid);
    d.mem_limit = resolved.dev[i].mem_limit;
    d.hbm_limit = 0;
    d.cu_limit_pct = 0;
    d.gate_open.store(1);
    d.configured = 1;
    if (r->hdr.num_devices < i + 1) r->hdr.num_devices = i + 1;
  }
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    DeviceState& d = r->dev[i];
    if (d.configured) continue;
    snprintf(d.uuid, sizeof(d.uuid), "%.63s", a.uuid);  // UUIDs are "GPU-" + 16 hex digits
    d.phys_total = a.phys_total;
    d.cu_count = a.cu_count;
    d.num_xcc = a.num_xcc;
    d.gpu_id = a.gpu_id;
    VGPU_REAL_HSA(hsa_agent_get_info);
    uint32_t bdf = 0, dom = 0;
    real_hsa_agent_get_info(a.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
    real_hsa_agent_get_info(a.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
    d.bdf = bdf;
    d.domain = dom;
    if (per_agent[i].mem_limit) d.mem_limit = per_agent[i].mem_limit;
    if (per_agent[i].hbm_limit) d.hbm_limit = per_agent[i].hbm_limit;
    if (per_agent[i].cu_limit_pct) d.cu_limit_pct = per_agent[i].cu_limit_pct;
    if (per_agent[i].cu_range_begin >= 0) {
      d.cu_range_begin = per_agent[i].cu_range_begin;
      d.cu_range_end = per_agent[i].cu_range_end;
    }
    const char* layout = getenv("VGPU_CU_LAYOUT");  // "se" (default) | "interleave"
    d.num_se = (layout && !strcasecmp(layout, "interleave")) ? 1 : a.num_se;
    CuMask m = cu_mask_for(a.cu_count, a.num_xcc, d.cu_limit_pct, d.cu_range_begin, d.cu_range_end, d.num_se);
    memcpy(d.cu_mask, m.words, sizeof(d.cu_mask));
    d.cu_mask_bits = m.nbits;
    d.credit_ns.store(timeshare_params(d.cu_limit_pct, config().limiter_window_ms, d.cu_share_bp).burst_ns);
    d.gate_open.store(1);
    d.configured = 1;
  }
}

}  // namespace

int agent_ordinal(hsa_agent_t a) {
  ShimState& s = shim();
  for (int i = 0; i < s.n_agents; i++)
    if (s.agents[i].agent.handle == a.handle) return i;
  return -1;
}

int pool_ordinal(hsa_amd_memory_pool_t p) {
  ShimState& s = shim();
  for (int i = 0; i < s.n_agents; i++)
    for (int j = 0; j < s.agents[i].n_pools; j++)
      if (s.agents[i].pools[j].handle == p.handle) return i;
  return -1;
}

bool shim_attach_region_only() {
  ShimState& s = shim();
  if (s.region.attached()) return true;
  static std::once_flag once;
  std::call_once(once, [] {
    load_env_config();
    const Config& cfg = config();
    if (cfg.disabled) return;
    shim().region.attach(cfg.shared_cache.c_str(), &cfg, true);
  });
  return s.region.attached();
}

void shim_init_after_hsa() {
  ShimState& s = shim();
  int expected = 0;
  if (!s.phase.compare_exchange_strong(expected, 1)) {
    while (s.phase.load() == 1) {
      struct timespec ts = {0, 1000000};
      nanosleep(&ts, nullptr);
    }
    return;
  }
  s.pid = getpid();
  load_env_config();
  const Config& cfg = config();
  if (cfg.disabled) {
    s.phase.store(3);
    return;
  }

  AgentScan sc{&s, {}, 0};
  s.n_agents = 0;
  VGPU_REAL_HSA(hsa_iterate_agents);
  if (real_hsa_iterate_agents) real_hsa_iterate_agents(agent_cb, &sc);
  s.n_cpu_pools = 0;
  for (int c = 0; c < sc.n_cpu; c++) {
    VGPU_REAL_HSA(hsa_amd_agent_iterate_memory_pools);
    real_hsa_amd_agent_iterate_memory_pools(sc.cpus[c], cpu_pool_record_cb, &s);
  }
  // A GPU agent's region list (legacy API) also names the system memory regions it can reach
  // - the CPU pools under another name: host memory, not the GPU's (measured on MI355X: a
  // CPU-pool allocation was charged to the device quota, profiles/r5b).
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    int kept = 0;
    for (int j = 0; j < a.n_pools; j++) {
      bool host = false;
      for (int c = 0; c < s.n_cpu_pools && !host; c++) host = s.cpu_pools[c].handle == a.pools[j].handle;
      if (!host) a.pools[kept++] = a.pools[j];
    }
    a.n_pools = kept;
  }
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    if (!a.cpu_agent.handle && sc.n_cpu) a.cpu_agent = sc.cpus[0];
    if (a.cpu_agent.handle) {
      VGPU_REAL_HSA(hsa_amd_agent_iterate_memory_pools);
      real_hsa_amd_agent_iterate_memory_pools(a.cpu_agent, cpu_pool_cb, &a);
    }
  }

  // Resolve the vGPU map onto the visible agents.
  char uuids[kMaxDevices][64];
  const char* uuid_ptrs[kMaxDevices];
  VGPU_REAL_HSA(hsa_agent_get_info);
  for (int i = 0; i < s.n_agents; i++) {
    uuids[i][0] = 0;
    real_hsa_agent_get_info(s.agents[i].agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_UUID, uuids[i]);
    uuids[i][63] = 0;
    uuid_ptrs[i] = uuids[i];
  }
  for (int i = 0; i < s.n_agents; i++) memcpy(s.agents[i].uuid, uuids[i], sizeof(s.agents[i].uuid));
  DeviceMap map;
  const char* map_env = cfg.device_map.empty() ? nullptr : cfg.device_map.c_str();
  if (!parse_device_map(map_env, &map)) {
    VLOG_WARN("invalid VGPU_DEVICE_MAP=%s, using positional limits", map_env);
    map = DeviceMap();
  }
  // Device authorisation (reference: vgpuvalidator, dormant there): with VGPU_ALLOWLIST
  // set, GPUs whose ROCr UUID is not listed get no device memory at all.
  if (!cfg.allowlist.empty()) {
    const char* al = cfg.allowlist.c_str();
    if (FILE* f = fopen(al, "r")) {
      std::vector<std::string> allowed;
      char line[128];
      while (fgets(line, sizeof(line), f)) {
        char norm[64];
        line[strcspn(line, "\r\n")] = 0;
        normalize_uuid(line, norm, sizeof(norm));
        if (norm[0]) allowed.emplace_back(norm);
      }
      fclose(f);
      for (int i = 0; i < s.n_agents; i++) {
        char norm[64];
        normalize_uuid(uuids[i], norm, sizeof(norm));
        s.agents[i].authorised = std::find(allowed.begin(), allowed.end(), std::string(norm)) != allowed.end();
        if (!s.agents[i].authorised) VLOG_ERROR("device %d (%s) is not authorised for this container", i, uuids[i]);
      }
    } else {
      VLOG_WARN("VGPU_ALLOWLIST=%s is not readable; device authorisation skipped", al);
    }
  }
  Config resolved = cfg;
  DeviceConfig per_agent[kMaxDevices];
  resolve_devices(cfg, map, uuid_ptrs, s.n_agents, per_agent);
  for (int i = 0; i < s.n_agents; i++) {
    if (!per_agent[i].unmapped) continue;
    s.agents[i].authorised = false;
    VLOG_ERROR("device %d (%s) is not in VGPU_DEVICE_MAP: no device memory for it in this container", i, uuids[i]);
  }
  for (int i = 0; i < kMaxDevices; i++) resolved.dev[i] = i < s.n_agents ? per_agent[i] : DeviceConfig();
  resolved.num_devices = s.n_agents;
  if (cfg.duplicate_split && map.duplicates) {
    // Split duplicate vGPUs (vdev_hooks.cpp): each vGPU of a GPU that backs several gets a
    // region slot of its own after the agents' - agent by agent, in map order - holding its
    // quota; the agent's slot keeps the summed quota as the physical guard.
    int next = s.n_agents;
    for (int a = 0; a < s.n_agents; a++) {
      char au[64];
      normalize_uuid(uuids[a], au, sizeof(au));
      int idx[kMaxDevices], c = 0;
      for (int j = 0; j < map.n; j++) {
        char mu[64];
        normalize_uuid(map.e[j].uuid, mu, sizeof(mu));
        if (!strcmp(mu, au)) idx[c++] = map.e[j].vidx;
      }
      for (int k = 0; c > 1 && k < c && next < kMaxDevices; k++, next++) {
        DeviceConfig v = cfg.dev[idx[k]];
        v.cu_limit_pct = 0;  // compute stays per physical GPU (the agent's slot)
        v.cu_range_begin = v.cu_range_end = -1;
        memcpy(v.uuid, uuids[a], sizeof(v.uuid) - 1);
        v.uuid[sizeof(v.uuid) - 1] = 0;
        resolved.dev[next] = v;
      }
    }
    resolved.num_devices = next;
    VLOG_INFO("duplicate vGPUs split: %d virtual quota slot(s)", next - s.n_agents);
  }

  // Host PID: sysfs is not PID-namespaced; outside a container it equals getpid(),
  // inside one the VRAM signature resolves it (the maintenance thread retries).
  if (!s.hostpid) s.hostpid = resolve_hostpid(2000);

  install_ceilings(uuid_ptrs);
  s.resolved = resolved;
  int rc = s.region.attach(cfg.shared_cache.c_str(), &resolved, true);
  if (rc == -ENOENT) {
    // The region's directory is missing (e.g. a monitor-mode host directory removed under
    // a running pod): recreate it, so this container keeps one region.
    std::string dir = cfg.shared_cache.substr(0, cfg.shared_cache.rfind('/'));
    for (size_t i = 1; i <= dir.size(); i++)
      if (i == dir.size() || dir[i] == '/') mkdir(dir.substr(0, i).c_str(), 0755);
    rc = s.region.attach(cfg.shared_cache.c_str(), &resolved, true);
  }
  if (rc == 0 && cfg.region_inode && s.region.inode() != cfg.region_inode) {
    // Not the region file the plugin created for this container (deleted and re-created,
    // or the path pointed elsewhere): its accounting is not the container's.
    VLOG_ERROR("shared region %s is not the plugin's (inode %lu, expected %lu)", cfg.shared_cache.c_str(),
               (unsigned long)s.region.inode(), (unsigned long)cfg.region_inode);
    s.region.detach();
    rc = -EPERM;
  }
  if (rc != 0) {
    // Without the region there is no shared accounting. With limits configured the shim
    // fails closed - no device memory - rather than letting the container run unlimited
    // (VGPU_FAIL_OPEN=1 restores the pass-through).
    s.fail_closed = !cfg.fail_open && (cfg.any_memory_limit() || cfg.any_cu_limit() || s.has_ceiling);
    VLOG_ERROR("cannot attach shared region %s (%s); %s", cfg.shared_cache.c_str(), strerror(-rc),
               s.fail_closed ? "device memory is refused (fail closed)" : "limits are NOT enforced");
    s.phase.store(3);
    return;
  }
  Region* r = s.region.raw();
  s.region.lock();
  configure_devices(r, per_agent, resolved);
  s.region.unlock();
  clamp_region_to_ceiling();
  s.seen_generation.store(r->hdr.generation.load() - 1);  // forces the first apply below
  apply_live_config();

  s.epoch = r->hdr.epoch;
  s.slot = s.region.register_process(s.pid, s.hostpid, cfg.priority);
  s.active = s.slot >= 0;
  if (cfg.signal_control) {
    signal(SIGUSR2, on_signal_suspend);
    signal(SIGUSR1, on_signal_resume);
  }
  static std::once_flag hooks_once;
  std::call_once(hooks_once, [] {
    pthread_atfork(atfork_prepare, atfork_parent, atfork_child);
    atexit(on_exit);
  });
  for (int i = 0; i < s.n_agents; i++) {
    const DeviceState& d = r->dev[i];
    VLOG_INFO("device %d uuid=%s gpu_id=%u cus=%d xcc=%d limit=%lu MiB cu_limit=%d%% mask=%d CUs%s%s hostpid=%d", i,
              d.uuid, s.agents[i].gpu_id, s.agents[i].cu_count, s.agents[i].num_xcc,
              (unsigned long)(d.mem_limit >> 20), d.cu_limit_pct, s.agents[i].mask.count(),
              s.agents[i].mask_active ? " [spatial]" : "", s.agents[i].temporal_active ? " [temporal]" : "",
              (int)s.hostpid);
  }
  s.phase.store(2);
  start_watcher_if_needed();
}

namespace {

bool probe_vram(void* ctx, uint64_t bytes, bool alloc) {
  // One probe buffer at a time (kfd_resolve_hostpid allocates, reads sysfs, frees).
  static void* ptr = nullptr;
  AgentInfo* a = static_cast<AgentInfo*>(ctx);
  if (alloc) {
    VGPU_REAL_HSA(hsa_amd_memory_pool_allocate);
    ptr = nullptr;
    return real_hsa_amd_memory_pool_allocate(a->vram_pool, bytes, 0, &ptr) == HSA_STATUS_SUCCESS && ptr;
  }
  VGPU_REAL_HSA(hsa_amd_memory_pool_free);
  if (ptr) real_hsa_amd_memory_pool_free(ptr);
  ptr = nullptr;
  return true;
}

}  // namespace

pid_t resolve_hostpid(int lock_timeout_ms) {
  ShimState& s = shim();
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    if (!a.gpu_id || !a.vram_pool.handle) continue;
    return kfd_resolve_hostpid(a.gpu_id, probe_vram, &a, config().lock_file.c_str(), lock_timeout_ms,
                               (unsigned)(now_ns() ^ (uint64_t)getpid() << 20));
  }
  std::vector<int> pids = kfd_list_pids();
  return std::binary_search(pids.begin(), pids.end(), (int)getpid()) ? getpid() : 0;
}

bool clamp_region_to_ceiling() {
  ShimState& s = shim();
  if (!s.has_ceiling || !s.region.attached()) return false;
  Region* r = s.region.raw();
  bool clamped = false;
  const bool locked = s.region.lock_for(kLockTimeoutMs);
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    DeviceState& d = r->dev[i];
    const uint64_t cm = s.region.ceiling(i);
    if (cm && (!d.mem_limit || d.mem_limit > cm)) {
      VLOG_WARN("device %d: region memory limit %lu above the plugin's %lu; clamped", i, (unsigned long)d.mem_limit,
                (unsigned long)cm);
      d.mem_limit = cm;
      clamped = true;
    }
    const uint64_t ch = s.region.hbm_ceiling(i);
    if (ch && (!d.hbm_limit || d.hbm_limit > ch)) {
      VLOG_WARN("device %d: region HBM share %lu above the plugin's %lu; clamped", i, (unsigned long)d.hbm_limit,
                (unsigned long)ch);
      d.hbm_limit = ch;
      clamped = true;
    }
    if (a.ceil_pct > 0) {
      if (d.cu_limit_pct <= 0 || d.cu_limit_pct >= 100 || d.cu_limit_pct > a.ceil_pct) {
        VLOG_WARN("device %d: region CU limit %d%% above the plugin's %d%%; clamped", i, d.cu_limit_pct, a.ceil_pct);
        d.cu_limit_pct = a.ceil_pct;
        clamped = true;
      }
      // The exact share the GPU-time grants use (with the node ledger) is a limit too: the
      // grant basis (the share, or the whole-percent limit when it is 0) may not exceed the
      // file's share nor the region's (possibly lowered) limit.
      const int pct_bp = d.cu_limit_pct * 100;
      const int limit_bp = std::min(a.ceil_share_bp, pct_bp);
      int share = d.cu_share_bp;
      if ((share > 0 ? share : pct_bp) > limit_bp) share = limit_bp == pct_bp ? 0 : limit_bp;
      if (share != d.cu_share_bp) {
        VLOG_WARN("device %d: region GPU-time share %d bp outside the plugin's %d bp; clamped", i, d.cu_share_bp,
                  a.ceil_share_bp);
        d.cu_share_bp = share;
        clamped = true;
      }
      // The slice may be narrowed live (set_cu_limit), never moved onto other CUs or widened.
      CuMask m;
      memcpy(m.words, d.cu_mask, sizeof(m.words));
      m.nbits = d.cu_mask_bits ? d.cu_mask_bits : a.cu_count;
      bool subset = m.count() > 0;
      for (int w = 0; w < kCuMaskWords && subset; w++) subset = (m.words[w] & ~a.ceil_mask.words[w]) == 0;
      if (!subset) {
        VLOG_WARN("device %d: region CU mask outside the plugin's slice; reset to it", i);
        memcpy(d.cu_mask, a.ceil_mask.words, sizeof(d.cu_mask));
        d.cu_mask_bits = a.ceil_mask.nbits;
        clamped = true;
      }
    }
  }
  const Config& cfg = config();
  if (cfg.host_mem_limit && (!r->hdr.host_limit || r->hdr.host_limit > cfg.host_mem_limit)) {
    r->hdr.host_limit = cfg.host_mem_limit;
    clamped = true;
  }
  if (r->hdr.priority.load(std::memory_order_relaxed) < cfg.min_priority) {
    r->hdr.priority.store(cfg.min_priority, std::memory_order_relaxed);
    clamped = true;
  }
  if (locked) s.region.unlock();
  return clamped;
}

void check_region_epoch() {
  ShimState& s = shim();
  if (!s.active || !s.region.attached() || s.exiting.load()) return;
  Region* r = s.region.raw();
  const bool reinit = s.region.reinit_if_invalid(&s.resolved);
  const bool moved = r->hdr.epoch != s.epoch;
  const bool lost = s.slot < 0 || r->procs[s.slot].pid.load(std::memory_order_relaxed) != s.pid;
  if (!reinit && !moved && !lost) return;
  VLOG_ERROR("shared region %s lost this process's slot (%s); registering and charging %s again",
             s.region.path(), reinit ? "overwritten" : moved ? "re-initialised" : "slot cleared", "its allocations");
  if (reinit || moved) {
    s.region.lock();
    DeviceConfig per_agent[kMaxDevices];
    for (int i = 0; i < kMaxDevices; i++) per_agent[i] = s.resolved.dev[i];
    configure_devices(r, per_agent, s.resolved);
    s.region.unlock();
    clamp_region_to_ceiling();
  }
  s.epoch = r->hdr.epoch;
  const int slot = s.region.register_process(s.pid, s.hostpid, config().priority);
  if (slot < 0) return;
  s.slot = slot;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    uint64_t host = 0;
    for (const auto& kv : s.allocs) {
      s.region.force_charge(slot, kv.second.dev, kv.second.size, (MemKind)kv.second.kind);
      if (kv.second.kind == kMemSpill) host += kv.second.size;  // spills are pinned host memory too
    }
    for (const auto& kv : s.vmem) s.region.force_charge(slot, kv.second.dev, kv.second.size, kMemData);
    for (const auto& kv : s.managed) s.region.force_charge(slot, kv.second.dev, kv.second.size, kMemData);
    host += host_recorded_bytes();
    svm_recharge(slot, &host);
    if (host) {
      r->hdr.host_used.fetch_add(host);
      r->procs[slot].host_used.fetch_add(host);
    }
  }
  svm_tenant_recharge(slot);
  resync_context_charge();
  r->hdr.generation.fetch_add(1, std::memory_order_acq_rel);  // every process re-applies its masks
}

void apply_live_config() {
  ShimState& s = shim();
  std::lock_guard<std::mutex> g(s.live_mu);
  Region* r = s.region.raw();
  const uint64_t gen = r->hdr.generation.load(std::memory_order_acquire);
  if (gen == s.seen_generation.load()) return;
  clamp_region_to_ceiling();
  const Config& cfg = config();
  const bool force = cfg.cu_policy == CuPolicy::kForce, off = cfg.cu_policy == CuPolicy::kDisable;
  for (int i = 0; i < s.n_agents; i++) {
    AgentInfo& a = s.agents[i];
    DeviceState& d = r->dev[i];
    // Bounded wait: this runs from the launch path, which must not hang behind a region
    // lock holder that is stopped; without the lock the read may see a half-written mask,
    // which the writer's generation bump makes every process re-read.
    const bool locked = s.region.lock_for(kLockTimeoutMs);
    CuMask m;
    memcpy(m.words, d.cu_mask, sizeof(m.words));
    m.nbits = d.cu_mask_bits ? d.cu_mask_bits : a.cu_count;
    const int pct = d.cu_limit_pct;
    const bool ranged = d.cu_range_begin >= 0;
    if (locked) s.region.unlock();
    const bool limited = pct > 0 && pct < 100;
    const int prio = effective_priority(r);
    // A thin slice (a few CUs per XCD) is no place for stock libraries' grids: in auto mode
    // such a share is time-sliced on every CU whatever the crowd, and the runtime is told the
    // whole GPU (profiles/r4c, r4g: 16 pods). The latency class keeps its slice.
    const bool thin = cfg.cu_mode == CuMode::kAuto && limited && prio > 0 && cfg.auto_min_slice_cus > 0 &&
                      m.count() > 0 && m.count() < cfg.auto_min_slice_cus;
    const CuMode mode =
        thin ? CuMode::kTemporal : effective_cu_mode_prio(cfg.cu_mode, pct, d.crowd.load(std::memory_order_relaxed), prio);
    const bool spatial = mode == CuMode::kSpatial || mode == CuMode::kBoth;
    const bool temporal = mode == CuMode::kTemporal || mode == CuMode::kBoth;
    const bool mask_on = !off && spatial && (limited || ranged) && m.count() < a.cu_count && m.count() > 0;
    // A background tenant is gated in time even without a share: it yields to busier
    // higher-priority tenants (watcher.cpp) and otherwise runs free.
    const bool yields = prio >= kPrioBackground && cfg.cu_mode == CuMode::kAuto && temporal;
    const bool temp_on = !off && temporal && (limited || force || yields);
    // A background tenant keeps its queues off the CUs latency-class tenants hold on this
    // GPU (their slices from the board, watcher.cpp): its work can then not sit in front
    // of theirs on a CU, whatever it has queued.
    bool reserved_on = false;
    if (!off && prio >= kPrioBackground) {
      CuMask rsv;
      memcpy(rsv.words, d.reserved_mask, sizeof(rsv.words));
      rsv.nbits = a.cu_count;
      // At most half the GPU can be held this way: the board is written by the tenants,
      // and one that claims more is ignored rather than allowed to starve this one.
      if (rsv.count() > 0 && rsv.count() <= a.cu_count / 2) {
        CuMask left;
        left.nbits = a.cu_count;
        for (int b = 0; b < a.cu_count && b < kMaxCUs; b++)
          if ((mask_on ? m.test(b) : true) && !rsv.test(b)) left.set(b);
        if (left.count() > 0 && cu_mask_balanced(left, a.num_xcc)) {
          m = left;
          reserved_on = true;
        }
      }
    }
    const bool mask_eff = mask_on || reserved_on;
    const bool mask_changed = mask_eff != a.mask_active.load() || memcmp(m.words, a.mask.words, sizeof(m.words)) != 0;
    if (temp_on && !a.temporal_active.load() && !d.gate_open.load()) {
      d.credit_ns.store(timeshare_params(pct, cfg.limiter_window_ms, d.cu_share_bp).burst_ns);
      d.gate_open.store(1);
    }
    a.mask = m;
    a.mode = mode;
    // Libraries size grids and pick kernels from the CU count (hipDeviceProp
    // multiProcessorCount, which CLR reads once from the agent): a vGPU with a CU slice
    // reports the slice, so stock MIOpen / hipBLASLt / PyTorch launches — cooperative and
    // persistent grids in particular — fit the CUs it may get. In auto mode the slice is
    // reported whether or not the mask is on at this moment, so every process of the
    // container sees the same count however crowded the GPU was when it started.
    const bool may_mask = spatial || (cfg.cu_mode == CuMode::kAuto && !thin);
    const bool slice = !off && may_mask && (limited || ranged) && m.count() < a.cu_count && m.count() > 0;
    a.visible_cus.store(slice && cfg.virtual_cu_count ? m.count() : 0);
    // Leaving the GPU-time limiter (auto mode: the GPU calmed down; a live share change):
    // nobody samples this device's credit any more, so a closed gate would never re-open
    // and a launch blocked on it would wait forever. Open it.
    if (!temp_on && !d.gate_open.load()) d.gate_open.store(1);
    a.temporal_active.store(temp_on);
    int flags = (mask_eff ? 1 : 0) | (temp_on ? 2 : 0);
    d.cu_mode.store(flags);
    if (mask_changed) {
      a.mask_active.store(mask_eff);
      // Re-apply to every queue this process already owns (they were created with the
      // old mask); new queues pick the mask up in hsa_queue_create.
      std::vector<hsa_queue_t*> qs;
      {
        std::lock_guard<std::mutex> q(s.queue_mu);
        for (auto& kv : s.queues)
          if (kv.second == i) qs.push_back(reinterpret_cast<hsa_queue_t*>(kv.first));
      }
      VGPU_REAL_HSA(hsa_amd_queue_cu_set_mask);
      CuMask all;
      for (int b = 0; b < a.cu_count && b < kMaxCUs; b++) all.set(b);
      const CuMask& eff = mask_eff ? m : all;
      uint32_t nbits = (uint32_t)((a.cu_count + 31) / 32 * 32);
      for (hsa_queue_t* q : qs) {
        hsa_status_t st = real_hsa_amd_queue_cu_set_mask(q, nbits, eff.words);
        if (st != HSA_STATUS_SUCCESS && (int)st != (int)HSA_STATUS_CU_MASK_REDUCED)
          VLOG_ERROR("device %d: cannot re-apply CU mask to queue %p (status %d)", i, (void*)q, (int)st);
      }
      if (!qs.empty())
        VLOG_INFO("device %d: CU limit %d%%%s -> %d CUs re-applied to %zu queue(s)", i, pct,
                  reserved_on ? " (off the latency class's CUs)" : "", mask_eff ? m.count() : a.cu_count, qs.size());
    }
  }
  bool any = false;
  for (int i = 0; i < s.n_agents; i++) any |= s.agents[i].temporal_active.load();
  s.any_temporal.store(any);
  s.seen_generation.store(gen);
  if (s.phase.load() == 2) start_watcher_if_needed();
}

void resync_context_charge() {
  ShimState& s = shim();
  if (!s.active || s.slot < 0 || !s.hostpid || s.exiting.load()) return;
  // Called from hsa_queue_create and the maintenance thread: both would compute the same
  // delta from the same ctx_had and charge it twice (a spurious OOM near the quota).
  std::lock_guard<std::mutex> g(s.ctx_mu);
  Region* r = s.region.raw();
  for (int i = 0; i < s.n_agents; i++) {
    const AgentInfo& a = s.agents[i];
    if (!a.gpu_id) continue;
    int64_t vram = kfd_vram_usage(s.hostpid, a.gpu_id);
    if (vram < 0) continue;
    DeviceUsage& u = r->procs[s.slot].used[i];
    // Promoted SVM spills and the tenant's own SVM ranges are charged as data; KFD may not
    // count their pages in vram_<id>.
    int64_t tracked = (int64_t)u.kind[kMemData].load() - svm_hbm_outside_kfd(i) - svm_tenant_outside_kfd(i);
    // IPC imports are not in the importer's vram_<gpu_id> (measured on MI355X: a 1 GiB
    // import left the consumer's counter at its ~0.5 GiB runtime footprint,
    // profiles/r2e), so nothing is subtracted for them: the exporter alone holds the charge.
    int64_t ctx_now = vram - tracked;
    if (ctx_now < 0) ctx_now = 0;
    int64_t ctx_had = (int64_t)u.kind[kMemContext].load();
    if (ctx_now > ctx_had) s.region.force_charge(s.slot, i, (uint64_t)(ctx_now - ctx_had), kMemContext);
    else if (ctx_now < ctx_had) s.region.uncharge(s.slot, i, (uint64_t)(ctx_had - ctx_now), kMemContext);
  }
}

void gate_suspend_slow() {
  ShimState& s = shim();
  uint64_t t0 = now_ns();
  bool logged = false;
  struct timespec ts = {0, 1000000};
  trace_push("vgpu:suspended");
  while (gate_needed()) {
    if (!logged) {
      VLOG_INFO("process suspended by controller; waiting");
      logged = true;
    }
    nanosleep(&ts, nullptr);
  }
  trace_pop();
  if (s.slot >= 0) s.region.raw()->procs[s.slot].suspend_ns.fetch_add(now_ns() - t0);
}

}  // namespace vgpu
