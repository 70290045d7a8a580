// Env contract parser (see vgpu/config.h for the reference mapping).
#include "vgpu/config.h"

#include <algorithm>
#include <cerrno>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <utility>
#include <vector>

#include <unistd.h>

#include "vgpu/log.h"

namespace vgpu {

namespace {
// Never destroyed: the shim's maintenance thread and hooks the runtime calls during its
// own teardown read the configuration after static destructors have started to run.
Config& g_config = *new Config();

bool parse_bool(const char* s, bool dflt) {
  if (!s || !*s) return dflt;
  if (!strcasecmp(s, "1") || !strcasecmp(s, "true") || !strcasecmp(s, "yes") || !strcasecmp(s, "on"))
    return true;
  if (!strcasecmp(s, "0") || !strcasecmp(s, "false") || !strcasecmp(s, "no") || !strcasecmp(s, "off"))
    return false;
  return dflt;
}

bool parse_int(const char* s, long lo, long hi, long* out) {
  if (!s || !*s) return false;
  char* end = nullptr;
  errno = 0;
  long v = strtol(s, &end, 10);
  if (errno || end == s) return false;
  while (*end == ' ' || *end == '%') end++;
  if (*end) return false;
  if (v < lo || v > hi) return false;
  *out = v;
  return true;
}
}  // namespace

CuMode effective_cu_mode(CuMode m, int pct, int crowd) {
  if (m != CuMode::kAuto) return m;
  if (pct <= 0 || pct >= 100) return CuMode::kSpatial;  // unlimited: no mask is applied anyway
  if (pct >= kAutoSpatialMinPct) return CuMode::kSpatial;
  return crowd >= 0 && crowd <= kAutoSpatialMaxCrowd ? CuMode::kSpatial : CuMode::kTemporal;
}

CuMode effective_cu_mode_prio(CuMode m, int pct, int crowd, int priority) {
  const CuMode base = effective_cu_mode(m, pct, crowd);
  if (m != CuMode::kAuto) return base;
  if (priority <= 0) return CuMode::kSpatial;
  if (priority >= 2 && crowd != 0) return CuMode::kTemporal;
  return base;
}

uint64_t spill_reserve(const Config& cfg, uint64_t hbm_share) {
  if (cfg.spill_reserve_bytes) return cfg.spill_reserve_bytes;
  const uint64_t floor = std::min<uint64_t>(2ull << 30, hbm_share / 4);
  return std::max<uint64_t>(floor, hbm_share / 16);
}

uint64_t spill_small_headroom(const Config& cfg, uint64_t hbm_share) {
  if (cfg.spill_small_headroom >= 0) return (uint64_t)cfg.spill_small_headroom;
  return std::min<uint64_t>(1ull << 30, hbm_share / 64);
}

bool Config::any_memory_limit() const {
  for (int i = 0; i < kMaxDevices; i++)
    if (dev[i].mem_limit) return true;
  return false;
}

bool Config::any_cu_limit() const {
  for (int i = 0; i < kMaxDevices; i++)
    if (dev[i].cu_limit_pct > 0 && dev[i].cu_limit_pct < 100) return true;
  return false;
}

bool parse_size(const char* s, uint64_t* out) {
  if (!s) return false;
  while (*s == ' ') s++;
  if (!*s || *s == '-') return false;
  char* end = nullptr;
  errno = 0;
  unsigned long long v = strtoull(s, &end, 10);
  if (errno || end == s) return false;
  unsigned shift = 0;
  switch (*end) {
    case 'k': case 'K': shift = 10; end++; break;
    case 'm': case 'M': shift = 20; end++; break;
    case 'g': case 'G': shift = 30; end++; break;
    case 't': case 'T': shift = 40; end++; break;
    case 0: break;
    default:
      if (*end != 'b' && *end != 'B') return false;
  }
  if (shift && (*end == 'i')) end++;
  if (*end == 'b' || *end == 'B') end++;
  while (*end == ' ') end++;
  if (*end) return false;
  if (shift && v > (~0ULL >> shift)) return false;  // overflow (reference rejects too)
  *out = (uint64_t)(v << shift);
  return true;
}

bool parse_range(const char* s, int* begin, int* end) {
  if (!s || !*s) return false;
  int a = 0, b = 0;
  char sep = 0;
  if (sscanf(s, "%d%c%d", &a, &sep, &b) != 3) return false;
  if (sep == ':') b = a + b;
  else if (sep != '-') return false;
  if (a < 0 || b <= a || b > kMaxCUs) return false;
  *begin = a;
  *end = b;
  return true;
}

int apply_override_env_file(const char* path) {
  FILE* f = fopen(path, "r");
  if (!f) return 0;
  char line[1024];
  int n = 0;
  while (fgets(line, sizeof(line), f)) {
    size_t len = strlen(line);
    while (len && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
    char* p = line;
    while (*p == ' ' || *p == '\t') p++;
    if (!*p || *p == '#') continue;
    if (!strncmp(p, "export ", 7)) p += 7;
    char* eq = strchr(p, '=');
    if (!eq || eq == p) continue;
    *eq = 0;
    if (setenv(p, eq + 1, 1) == 0) n++;
  }
  fclose(f);
  return n;
}

namespace {
// Pod specs written for the reference set some shim knobs by hand; those names are
// accepted when the VGPU_* name is absent (the plugin itself only emits VGPU_* names).
struct Alias {
  const char* name;
  const char* legacy;
};
const Alias kAliases[] = {
    {"VGPU_DEVICE_MEMORY_LIMIT", "CUDA_DEVICE_MEMORY_LIMIT"},
    {"VGPU_DEVICE_CU_LIMIT", "CUDA_DEVICE_SM_LIMIT"},
    {"VGPU_SHARED_CACHE", "CUDA_DEVICE_MEMORY_SHARED_CACHE"},
    {"VGPU_OVERSUBSCRIBE", "CUDA_OVERSUBSCRIBE"},
    {"VGPU_TASK_PRIORITY", "CUDA_TASK_PRIORITY"},
    {"VGPU_CU_POLICY", "GPU_CORE_UTILIZATION_POLICY"},
    {"VGPU_ACTIVE_OOM_KILLER", "ACTIVE_OOM_KILLER"},
    {"VGPU_MEMORY_OVERRIDE", "MEMORY_OVERRIDE"},
};

struct Env {
  GetenvFn fn;
  const char* operator()(const char* key) const {
    if (const char* v = fn(key)) return v;
    for (const Alias& a : kAliases)
      if (!strcmp(key, a.name)) return fn(a.legacy);
    // per-device memory limits: VGPU_DEVICE_MEMORY_LIMIT_<i> <- CUDA_DEVICE_MEMORY_LIMIT_<i>
    static const char kMem[] = "VGPU_DEVICE_MEMORY_LIMIT_";
    if (!strncmp(key, kMem, sizeof(kMem) - 1)) {
      char legacy[128];
      snprintf(legacy, sizeof(legacy), "CUDA_DEVICE_MEMORY_LIMIT_%.64s", key + sizeof(kMem) - 1);
      return fn(legacy);
    }
    return nullptr;
  }
};
}  // namespace

void load_config(Config* cfg, GetenvFn raw_getenv) {
  if (!raw_getenv) raw_getenv = [](const char* k) -> const char* { return getenv(k); };
  const Env getenv_fn{raw_getenv};
  *cfg = Config();
  cfg->disabled = parse_bool(getenv_fn("VGPU_DISABLE"), false);

  uint64_t global_limit = 0;
  if (const char* s = getenv_fn("VGPU_DEVICE_MEMORY_LIMIT")) {
    if (!parse_size(s, &global_limit)) VLOG_WARN("invalid VGPU_DEVICE_MEMORY_LIMIT=%s ignored", s);
  }
  uint64_t global_hbm = 0;
  if (const char* s = getenv_fn("VGPU_DEVICE_HBM_LIMIT")) {
    if (!parse_size(s, &global_hbm)) VLOG_WARN("invalid VGPU_DEVICE_HBM_LIMIT=%s ignored", s);
  }
  long global_cu = 0;
  if (const char* s = getenv_fn("VGPU_DEVICE_CU_LIMIT")) {
    if (!parse_int(s, 0, 100, &global_cu)) {
      VLOG_WARN("invalid VGPU_DEVICE_CU_LIMIT=%s ignored", s);
      global_cu = 0;
    }
  }
  char key[96];
  int max_idx = -1;
  for (int i = 0; i < kMaxDevices; i++) {
    DeviceConfig& d = cfg->dev[i];
    d.mem_limit = global_limit;
    d.hbm_limit = global_hbm;
    d.cu_limit_pct = (int)global_cu;
    snprintf(key, sizeof(key), "VGPU_DEVICE_MEMORY_LIMIT_%d", i);
    if (const char* s = getenv_fn(key)) {
      uint64_t v = 0;
      if (parse_size(s, &v)) {
        d.mem_limit = v;
        max_idx = i > max_idx ? i : max_idx;
      } else {
        VLOG_WARN("invalid %s=%s ignored", key, s);
      }
    }
    snprintf(key, sizeof(key), "VGPU_DEVICE_HBM_LIMIT_%d", i);
    if (const char* s = getenv_fn(key)) {
      uint64_t v = 0;
      if (parse_size(s, &v)) d.hbm_limit = v;
      else VLOG_WARN("invalid %s=%s ignored", key, s);
    }
    snprintf(key, sizeof(key), "VGPU_DEVICE_CU_LIMIT_%d", i);
    if (const char* s = getenv_fn(key)) {
      long v = 0;
      if (parse_int(s, 0, 100, &v)) {
        d.cu_limit_pct = (int)v;
        max_idx = i > max_idx ? i : max_idx;
      } else {
        VLOG_WARN("invalid %s=%s ignored", key, s);
      }
    }
    snprintf(key, sizeof(key), "VGPU_DEVICE_CU_SHARE_%d", i);
    if (const char* s = getenv_fn(key)) {
      // A decimal percent ("6.25"): the exact share of a vGPU whose CU limit was rounded up.
      char* end = nullptr;
      const double v = strtod(s, &end);
      if (end != s && !*end && v > 0.0 && v <= 100.0) d.cu_share_bp = (int)(v * 100.0 + 0.5);
      else VLOG_WARN("invalid %s=%s ignored", key, s);
    }
    snprintf(key, sizeof(key), "VGPU_DEVICE_CU_RANGE_%d", i);
    if (const char* s = getenv_fn(key)) {
      if (!parse_range(s, &d.cu_range_begin, &d.cu_range_end)) {
        VLOG_WARN("invalid %s=%s ignored", key, s);
        d.cu_range_begin = d.cu_range_end = -1;
      }
    }
  }
  cfg->num_devices = max_idx + 1;

  if (const char* s = getenv_fn("VGPU_SHARED_CACHE")) {
    if (*s) cfg->shared_cache = s;
  }
  cfg->oversubscribe = parse_bool(getenv_fn("VGPU_OVERSUBSCRIBE"), false);
  if (const char* s = getenv_fn("VGPU_SPILL_POLICY")) {
    if (!strcasecmp(s, "first-come") || !strcasecmp(s, "fifo")) cfg->spill_policy = SpillPolicy::kFirstCome;
    else if (!strcasecmp(s, "large-first")) cfg->spill_policy = SpillPolicy::kLargeFirst;
    else VLOG_WARN("invalid VGPU_SPILL_POLICY=%s, using large-first", s);
  }
  if (const char* s = getenv_fn("VGPU_SPILL_LARGE")) {
    if (!parse_size(s, &cfg->spill_large_bytes)) VLOG_WARN("invalid VGPU_SPILL_LARGE=%s ignored", s);
  }
  if (const char* s = getenv_fn("VGPU_SPILL_RESERVE")) {
    if (!parse_size(s, &cfg->spill_reserve_bytes)) VLOG_WARN("invalid VGPU_SPILL_RESERVE=%s ignored", s);
  }
  if (const char* s = getenv_fn("VGPU_SPILL_SMALL")) {
    if (!parse_size(s, &cfg->spill_small_bytes)) VLOG_WARN("invalid VGPU_SPILL_SMALL=%s ignored", s);
  }
  if (const char* s = getenv_fn("VGPU_SPILL_SMALL_HEADROOM")) {
    uint64_t v = 0;
    if (parse_size(s, &v) && v <= (uint64_t)INT64_MAX) cfg->spill_small_headroom = (int64_t)v;
    else VLOG_WARN("invalid VGPU_SPILL_SMALL_HEADROOM=%s ignored", s);
  }
  if (const char* s = getenv_fn("VGPU_SPILL_BACKING")) {
    if (!strcasecmp(s, "auto")) cfg->spill_backing = SpillBacking::kAuto;
    else if (!strcasecmp(s, "svm")) cfg->spill_backing = SpillBacking::kSvm;
    else if (!strcasecmp(s, "pinned")) cfg->spill_backing = SpillBacking::kPinned;
    else VLOG_WARN("invalid VGPU_SPILL_BACKING=%s, using auto", s);
  }
  cfg->spill_promote = parse_bool(getenv_fn("VGPU_SPILL_PROMOTE"), true);
  {
    long ms = 0;
    if (parse_int(getenv_fn("VGPU_DEMOTE_WAIT_MS"), 0, 60000, &ms)) cfg->demote_wait_ms = (int)ms;
  }
  if (const char* s = getenv_fn("VGPU_HOST_MEMORY_LIMIT")) {
    if (!parse_size(s, &cfg->host_mem_limit)) {
      VLOG_WARN("invalid VGPU_HOST_MEMORY_LIMIT=%s ignored", s);
      cfg->host_mem_limit = 0;
    }
  }
  long prio = 1;
  if (parse_int(getenv_fn("VGPU_TASK_PRIORITY"), -1000, 1000, &prio)) cfg->priority = (int)prio;

  if (const char* s = getenv_fn("VGPU_CU_MODE")) {
    if (!strcasecmp(s, "spatial")) cfg->cu_mode = CuMode::kSpatial;
    else if (!strcasecmp(s, "temporal")) cfg->cu_mode = CuMode::kTemporal;
    else if (!strcasecmp(s, "both")) cfg->cu_mode = CuMode::kBoth;
    else if (!strcasecmp(s, "off") || !strcasecmp(s, "none")) cfg->cu_mode = CuMode::kOff;
    else if (!strcasecmp(s, "auto")) cfg->cu_mode = CuMode::kAuto;
    else VLOG_WARN("invalid VGPU_CU_MODE=%s, using auto", s);
  }
  if (const char* s = getenv_fn("VGPU_CU_POLICY")) {
    if (!strcasecmp(s, "force")) cfg->cu_policy = CuPolicy::kForce;
    else if (!strcasecmp(s, "disable")) cfg->cu_policy = CuPolicy::kDisable;
  }
  cfg->active_oom_killer = parse_bool(getenv_fn("VGPU_ACTIVE_OOM_KILLER"), true);  // reference: unset = on
  cfg->memory_override = parse_bool(getenv_fn("VGPU_MEMORY_OVERRIDE"), false);
  if (const char* s = getenv_fn("VGPU_SYNC_WAIT")) {
    if (!strcasecmp(s, "auto")) cfg->sync_wait = SyncWait::kAuto;
    else if (!strcasecmp(s, "poll")) cfg->sync_wait = SyncWait::kPoll;
    else if (!strcasecmp(s, "native") || !strcasecmp(s, "spin")) cfg->sync_wait = SyncWait::kNative;
    else VLOG_WARN("invalid VGPU_SYNC_WAIT=%s, using auto", s);
  }
  cfg->signal_control = parse_bool(getenv_fn("VGPU_SIGNAL_CONTROL"), false);
  cfg->fail_open = parse_bool(getenv_fn("VGPU_FAIL_OPEN"), false);
  cfg->hook_smi = parse_bool(getenv_fn("VGPU_HOOK_SMI"), true);
  cfg->virtual_cu_count = parse_bool(getenv_fn("VGPU_VIRTUAL_CU_COUNT"), true);
  long min_slice = 40;
  if (parse_int(getenv_fn("VGPU_AUTO_MIN_SLICE_CUS"), 0, 1024, &min_slice)) cfg->auto_min_slice_cus = (int)min_slice;
  long period = 120;
  if (parse_int(getenv_fn("VGPU_UTIL_PERIOD_MS"), 10, 10000, &period)) cfg->util_period_ms = (int)period;
  long sample = 1000;
  if (parse_int(getenv_fn("VGPU_UTIL_SAMPLE_US"), 200, 100000, &sample)) cfg->util_sample_us = (int)sample;
  long budget = 32;
  if (parse_int(getenv_fn("VGPU_SAMPLE_READ_BUDGET"), 0, 1 << 20, &budget)) cfg->sample_read_budget = (int)budget;
  long window = 40;
  if (parse_int(getenv_fn("VGPU_LIMITER_WINDOW_MS"), 5, 2000, &window)) cfg->limiter_window_ms = (int)window;
  long solo = 160;
  if (parse_int(getenv_fn("VGPU_LIMITER_SOLO_WINDOW_MS"), 0, 5000, &solo)) cfg->limiter_solo_window_ms = (int)solo;
  if (const char* s = getenv_fn("VGPU_CHARGE_MODEL")) {
    if (!strcasecmp(s, "share")) cfg->charge_model = ChargeModel::kShare;
    else if (!strcasecmp(s, "progress")) cfg->charge_model = ChargeModel::kProgress;
    else VLOG_WARN("invalid VGPU_CHARGE_MODEL=%s ignored", s);
  }
  if (const char* s = getenv_fn("VGPU_BOARD_DIR")) cfg->board_dir = s;
  long conc = 0;
  if (const char* c = getenv_fn("VGPU_GPU_CONCURRENCY"); c && !strcasecmp(c, "auto")) cfg->gpu_concurrency = -1;
  else if (parse_int(c, 0, 64, &conc)) cfg->gpu_concurrency = (int)conc;
  long pr = 0;
  if (parse_int(getenv_fn("VGPU_PAIRS_ON_RATE"), 1, 100000000, &pr)) cfg->pairs_on_rate = (uint32_t)pr;
  if (parse_int(getenv_fn("VGPU_PAIRS_OFF_RATE"), 0, 100000000, &pr)) cfg->pairs_off_rate = (uint32_t)pr;
  if (cfg->pairs_off_rate > cfg->pairs_on_rate) cfg->pairs_off_rate = cfg->pairs_on_rate;
  long slice = 20;
  if (parse_int(getenv_fn("VGPU_GPU_SLICE_MS"), 1, 10000, &slice)) cfg->gpu_slice_ms = (int)slice;
  if (const char* s = getenv_fn("VGPU_BOARD_SLOT")) cfg->board_slot = s;
  long cpu_node = -1;
  const char* spread = getenv_fn("VGPU_CPU_SPREAD");
  if (!(spread && spread[0] == '0') && parse_int(getenv_fn("VGPU_CPU_NODE"), 0, 63, &cpu_node))
    cfg->cpu_node = (int)cpu_node;
  if (const char* s = getenv_fn("VGPU_LEDGER")) cfg->use_ledger = !(s[0] == '0' && !s[1]);
  long hold = 3;
  if (parse_int(getenv_fn("VGPU_PREEMPT_HOLD_MS"), 0, 10000, &hold)) cfg->preempt_hold_ms = (int)hold;
  long depth = 4;
  if (parse_int(getenv_fn("VGPU_PREEMPT_DEPTH"), 0, 4096, &depth)) cfg->preempt_depth = (int)depth;
  long crowd_depth = 16;
  if (parse_int(getenv_fn("VGPU_CROWD_DEPTH"), 0, 65536, &crowd_depth)) cfg->crowd_depth = (int)crowd_depth;
  if (const char* s = getenv_fn("VGPU_LOCK_FILE")) {
    if (*s) cfg->lock_file = s;
  }
  long merge = 1;
  if (parse_int(getenv_fn("VGPU_DUPLICATE_MERGE"), 0, 1, &merge)) cfg->duplicate_merge = (int)merge;
  long split = 0;
  if (parse_int(getenv_fn("VGPU_DUPLICATE_SPLIT"), 0, 1, &split)) cfg->duplicate_split = (int)split;
  if (const char* s = getenv_fn("VGPU_DEVICE_MAP")) cfg->device_map = s;
  if (const char* s = getenv_fn("VGPU_ALLOWLIST")) cfg->allowlist = s;
  long minp = 0;
  if (parse_int(getenv_fn("VGPU_TASK_PRIORITY_MIN"), -1000, 1000, &minp)) cfg->min_priority = (int)minp;
  if (const char* s = getenv_fn("VGPU_REGION_INODE")) cfg->region_inode = strtoull(s, nullptr, 10);
}

namespace {
// The limits file being parsed (load_config takes a plain function pointer).
const std::vector<std::pair<std::string, std::string>>* g_ceiling_kv = nullptr;
const char* ceiling_getenv(const char* key) {
  if (!g_ceiling_kv) return nullptr;
  for (const auto& kv : *g_ceiling_kv)
    if (kv.first == key) return kv.second.c_str();
  return nullptr;
}

uint64_t min_limit(uint64_t want, uint64_t ceil) {  // 0 = unlimited on either side
  if (!ceil) return want;
  return want && want < ceil ? want : ceil;
}
}  // namespace

bool load_ceiling(const char* path, Config* out) {
  FILE* f = path && *path ? fopen(path, "r") : nullptr;
  if (!f) return false;
  std::vector<std::pair<std::string, std::string>> kv;
  char line[1024];
  while (fgets(line, sizeof(line), f)) {
    size_t len = strlen(line);
    while (len && (line[len - 1] == '\n' || line[len - 1] == '\r')) line[--len] = 0;
    char* p = line;
    while (*p == ' ' || *p == '\t') p++;
    if (!*p || *p == '#') continue;
    char* eq = strchr(p, '=');
    if (!eq || eq == p) continue;
    *eq = 0;
    kv.emplace_back(p, eq + 1);
  }
  fclose(f);
  g_ceiling_kv = &kv;
  load_config(out, ceiling_getenv);
  g_ceiling_kv = nullptr;
  // A limits file without a class floor still keeps the tenant out of the latency class:
  // only the plugin grants it (VGPU_TASK_PRIORITY_MIN=0).
  if (out->min_priority == -1000) out->min_priority = 1;
  out->ceiling = true;
  return true;
}

void apply_ceiling(Config* cfg, const Config& ceil) {
  for (int i = 0; i < kMaxDevices; i++) {
    DeviceConfig& d = cfg->dev[i];
    const DeviceConfig& c = ceil.dev[i];
    d.mem_limit = min_limit(d.mem_limit, c.mem_limit);
    d.hbm_limit = min_limit(d.hbm_limit, c.hbm_limit);
    if (c.cu_limit_pct > 0 && c.cu_limit_pct < 100) {
      const bool unlimited = d.cu_limit_pct <= 0 || d.cu_limit_pct >= 100;
      d.cu_limit_pct = unlimited || d.cu_limit_pct > c.cu_limit_pct ? c.cu_limit_pct : d.cu_limit_pct;
      d.cu_share_bp = c.cu_share_bp && (!d.cu_share_bp || d.cu_share_bp > c.cu_share_bp) ? c.cu_share_bp : d.cu_share_bp;
      // The CUs are the plugin's choice (disjoint slices per vGPU), not the tenant's.
      d.cu_range_begin = c.cu_range_begin;
      d.cu_range_end = c.cu_range_end;
    }
  }
  if (ceil.num_devices > cfg->num_devices) cfg->num_devices = ceil.num_devices;
  cfg->host_mem_limit = min_limit(cfg->host_mem_limit, ceil.host_mem_limit);
  // Where the container's accounting lives and which GPU each vGPU index names: one region
  // and one map for every process of the container, whatever a process's environment says.
  cfg->shared_cache = ceil.shared_cache;
  if (!ceil.device_map.empty()) cfg->device_map = ceil.device_map;
  if (!ceil.allowlist.empty()) cfg->allowlist = ceil.allowlist;
  // The board (and the node ledger in it) is the plugin's too: a board of the tenant's own
  // could carry a forged ledger with no charges.
  if (!ceil.board_dir.empty()) cfg->board_dir = ceil.board_dir;
  if (!ceil.board_slot.empty()) cfg->board_slot = ceil.board_slot;
  if (ceil.gpu_concurrency != 0) cfg->gpu_concurrency = ceil.gpu_concurrency;  // the node's admission
  cfg->cu_mode = ceil.cu_mode;
  cfg->oversubscribe = cfg->oversubscribe && ceil.oversubscribe;
  // The memory backstop is the plugin's (on unless its limits file turns it off).
  cfg->active_oom_killer = ceil.active_oom_killer;
  if (ceil.min_priority > cfg->min_priority) cfg->min_priority = ceil.min_priority;
  if (cfg->priority < cfg->min_priority) cfg->priority = cfg->min_priority;
  if (ceil.region_inode) cfg->region_inode = ceil.region_inode;
  // Switches that would lift enforcement are the operator's, not the tenant's.
  cfg->disabled = false;
  cfg->fail_open = false;
  cfg->use_ledger = true;  // the ledger's exact charges are not the tenant's to opt out of
  if (cfg->cu_policy == CuPolicy::kDisable) cfg->cu_policy = CuPolicy::kDefault;
  cfg->ceiling = true;
}

bool ceiling_present() {
  if (access(kLimitsPath, R_OK) == 0) return true;
  const char* p = getenv("VGPU_LIMITS_FILE");
  return p && *p && access(p, R_OK) == 0;
}

const Config& config() { return g_config; }
Config& mutable_config() { return g_config; }

}  // namespace vgpu
