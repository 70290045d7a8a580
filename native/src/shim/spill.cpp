// Virtual device memory that moves: spilled allocations live in host memory until the
// tenant's HBM share has room for them again, then they are promoted into HBM at the same
// address, contents intact.
//
// Reference: with CUDA_OVERSUBSCRIBE every allocation becomes managed memory
// (server.go:505-507 → libvgpu.so cuMemoryAllocate@0x32146, allocmode 0 →
// cuMemAllocManaged) and the UVM driver moves hot pages back into device memory on demand.
// MI355X has no recoverable GPU page faults on this pool (XNACK off), so nothing moves on
// access. What KFD does have without XNACK is shared virtual memory (SVM): an ordinary range
// of the process's host memory registered for a GPU (hsa_amd_svm_attributes_set) is mapped
// into the GPU's page table in place, and hsa_amd_svm_prefetch_async migrates it into VRAM
// and back. The driver performs the migration with the process's queues evicted around it
// and restores the mapping before they resume, so a kernel never sees a half-moved range
// and no user-level stop-the-world is needed (a VMM re-map could not give that guarantee
// for work already queued).
//
// Placement: a spill is an anonymous mapping (MADV_DONTFORK: a forked child neither shares
// nor copies it) registered for the owning GPU in place with host memory preferred; it is
// charged as spill to the device quota and to the container's host budget, like the pinned
// spill it replaces (VGPU_SPILL_BACKING=pinned keeps that: a host-pool allocation, reachable
// by the GPU, that never moves). Promotion: a per-process thread (started with the first SVM
// spill) checks every period - and at once when the process frees device memory - whether
// the oldest spills fit: under the tenant's HBM share (VGPU_DEVICE_HBM_LIMIT_<i>) less the
// large-first reserve, and in the GPU's free HBM less the same reserve (other tenants'
// allocations come first). A promoted spill is charged as HBM data and released from the
// host budget; a failed migration (the driver refused, HBM went to someone else) is undone
// and retried after a back-off.
//
// Node-wide (the node board, vgpu/board.h): ROCr's free-memory figure does not show SVM pages
// in VRAM (profiles/r4b), so every process publishes its promoted spills and prefetched ranges
// (region slot -> the container's sampler -> its board slot), and every container takes the
// other containers' off the free HBM it places, promotes and reports by (hidden_vram). A
// tenant refused HBM within its quota while co-tenants hold promoted spills on the GPU asks for
// it on the board; their migrators demote their youngest promoted spills back to host memory
// (contents intact, charged as spill again) and the refused allocation is retried
// (reclaim_peer_hbm) - the two-way movement the reference's UVM spill has.
#include <errno.h>
#include <pthread.h>
#include <sys/mman.h>
#include <time.h>
#include <unistd.h>

#include <algorithm>
#include <cstdlib>
#include <atomic>
#include <mutex>
#include <vector>

#include "real.h"
#include "shim.h"
#include "vgpu/kfd.h"
#include "vgpu/log.h"
#include "vgpu/ratelimit.h"

namespace vgpu {

namespace {

constexpr uint64_t kPromoteBytesPerTick = 8ull << 30;        // migrated per period at most
// One range's migration (VGPU_SPILL_MIGRATE_TIMEOUT_MS, default 60 s).
uint64_t migrate_timeout_ns() {
  static const uint64_t ns = [] {
    const char* v = getenv("VGPU_SPILL_MIGRATE_TIMEOUT_MS");
    const long ms = v && *v ? strtol(v, nullptr, 10) : 0;
    return ms > 0 ? (uint64_t)ms * 1'000'000ull : 60'000'000'000ull;
  }();
  return ns;
}
constexpr uint64_t kRetryBackoffNs = 10'000'000'000ull;      // after a failed promotion
constexpr uint64_t kDemoteBackoffNs = 30'000'000'000ull;     // a demoted spill stays in host memory
constexpr uint64_t kBlindProbeBytes = 64ull << 20;           // migrations that measure MEMORY_AVAIL

// Whether ROCr's free-memory figure (HSA_AMD_AGENT_INFO_MEMORY_AVAIL) leaves out SVM pages in
// VRAM: -1 not measured yet (assumed, as measured on MI355X), 1 it does, 0 it shows them.
std::atomic<int> g_avail_blind{-1};

uint64_t real_mem_avail(const AgentInfo& a) {
  VGPU_REAL_HSA(hsa_agent_get_info);
  uint64_t v = 0;
  if (!real_hsa_agent_get_info ||
      real_hsa_agent_get_info(a.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MEMORY_AVAIL, &v) != HSA_STATUS_SUCCESS)
    return 0;
  return v;
}

// This process's SVM bytes in the VRAM of `dev` (plain loads of fields ctx_mu guards: an
// aligned 64-bit load is never torn, and a momentarily stale value is harmless here).
uint64_t own_svm_vram(const ShimState& s, int dev) {
  return (uint64_t)std::max<int64_t>(0, s.svm_hbm[dev] + s.tsvm_loc[dev]);
}

std::atomic<uint64_t> g_seq{0};
std::atomic<bool> g_migrator{false};
std::atomic<bool> g_wake{false};  // device memory was freed: look again before the period ends

// The driver has SVM and ROCr exposes it (checked once per process).
bool svm_supported() {
  static std::once_flag once;
  static bool ok = false;
  std::call_once(once, [] {
    VGPU_REAL_HSA(hsa_system_get_info);
    VGPU_REAL_HSA(hsa_amd_svm_attributes_set);
    VGPU_REAL_HSA(hsa_amd_svm_attributes_get);
    VGPU_REAL_HSA(hsa_amd_svm_prefetch_async);
    VGPU_REAL_HSA(hsa_signal_create);
    VGPU_REAL_HSA(hsa_signal_destroy);
    VGPU_REAL_HSA(hsa_signal_wait_scacquire);
    bool b = false;
    ok = real_hsa_system_get_info && real_hsa_amd_svm_attributes_set && real_hsa_amd_svm_attributes_get &&
         real_hsa_amd_svm_prefetch_async && real_hsa_signal_create && real_hsa_signal_destroy &&
         real_hsa_signal_wait_scacquire &&
         real_hsa_system_get_info((hsa_system_info_t)HSA_AMD_SYSTEM_INFO_SVM_SUPPORTED, &b) == HSA_STATUS_SUCCESS && b;
    VLOG_INFO("virtual device memory: SVM ranges %s", ok ? "available (spills can be promoted into HBM)"
                                                         : "unavailable (spills are pinned host memory)");
  });
  return ok;
}

size_t page_round(size_t n) {
  const size_t pg = (size_t)sysconf(_SC_PAGESIZE);
  return (n + pg - 1) / pg * pg;
}

bool accessible(uint64_t a) {
  return a == HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE || a == HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE;
}

// An SVM range of `size` bytes the GPU of `dev` reaches in place, in host memory.
hsa_status_t svm_map(int dev, size_t size, void** ptr, size_t* mapped) {
  ShimState& s = shim();
  const AgentInfo& a = s.agents[dev];
  VGPU_REAL_HSA(hsa_amd_svm_attributes_set);
  VGPU_REAL_HSA(hsa_amd_svm_attributes_get);
  const size_t len = page_round(size);
  void* p = mmap(nullptr, len, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (p == MAP_FAILED) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  madvise(p, len, MADV_DONTFORK);
  hsa_amd_svm_attribute_pair_t attrs[2] = {{HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE, a.agent.handle},
                                           {HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION, a.cpu_agent.handle}};
  hsa_status_t st = real_hsa_amd_svm_attributes_set(p, len, attrs, 2);
  // Used by a kernel only once the driver reports the GPU's access (no access = a fault).
  hsa_amd_svm_attribute_pair_t q[1] = {{HSA_AMD_SVM_ATTRIB_ACCESS_QUERY, a.agent.handle}};
  if (st == HSA_STATUS_SUCCESS) st = real_hsa_amd_svm_attributes_get(p, len, q, 1);
  if (st == HSA_STATUS_SUCCESS && !accessible(q[0].attribute)) st = HSA_STATUS_ERROR_INVALID_AGENT;
  if (st != HSA_STATUS_SUCCESS) {
    munmap(p, len);
    return st;
  }
  *ptr = p;
  *mapped = len;
  return HSA_STATUS_SUCCESS;
}

// Outcome of one range's migration.
enum class Migration { kDone, kFailed, kPending };

// Migrates [p, p+len) to `agent` (a GPU or the CPU) and waits for the driver (bounded). A
// migration still in flight at the bound keeps its completion signal: ROCr's async thread
// signals it later, so it is left allocated (a few bytes) rather than destroyed under it.
Migration migrate(void* p, size_t len, hsa_agent_t agent) {
  VGPU_REAL_HSA(hsa_amd_svm_attributes_set);
  VGPU_REAL_HSA(hsa_amd_svm_prefetch_async);
  VGPU_REAL_HSA(hsa_signal_create);
  VGPU_REAL_HSA(hsa_signal_destroy);
  VGPU_REAL_HSA(hsa_signal_wait_scacquire);
  hsa_amd_svm_attribute_pair_t pref[1] = {{HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION, agent.handle}};
  if (real_hsa_amd_svm_attributes_set(p, len, pref, 1) != HSA_STATUS_SUCCESS) return Migration::kFailed;
  hsa_signal_t sig;
  if (real_hsa_signal_create(1, 0, nullptr, &sig) != HSA_STATUS_SUCCESS) return Migration::kFailed;
  if (real_hsa_amd_svm_prefetch_async(p, len, agent, 0, nullptr, sig) != HSA_STATUS_SUCCESS) {
    real_hsa_signal_destroy(sig);
    return Migration::kFailed;
  }
  const hsa_signal_value_t v =
      real_hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, migrate_timeout_ns(), HSA_WAIT_STATE_BLOCKED);
  if (v >= 1) return Migration::kPending;  // still in flight: the signal stays valid for ROCr
  real_hsa_signal_destroy(sig);
  return v == 0 ? Migration::kDone : Migration::kFailed;
}

// Promotes the SVM spills of `dev` that fit, oldest first; returns the bytes moved.
//
// The charge moves from spill to HBM data before the migration, atomically against the
// container's concurrent allocations (SharedRegion::promote_spill: resident bytes stay within
// the share less the reserve), and back if the driver refuses. ctx_mu is held only around
// the bookkeeping, never across the migration (up to a minute), so the maintenance thread's
// context re-sync and the container's sampler are not held up meanwhile.
uint64_t promote_device(int dev, uint64_t budget) {
  ShimState& s = shim();
  const Config& cfg = config();
  AgentInfo& a = s.agents[dev];
  // A co-tenant on this GPU is short of HBM (the container was asked to demote): nothing moves up.
  if (s.region.raw()->dev[dev].demote_want.load(std::memory_order_relaxed)) return 0;
  const uint64_t share = s.region.hbm_limit(dev);
  const uint64_t reserve = share ? spill_reserve(cfg, share) : 0;
  const uint64_t cap = share ? (share > reserve ? share - reserve : 1) : 0;
  std::vector<std::pair<uint64_t, uintptr_t>> order;  // (seq, ptr) of the spills in host memory
  const uint64_t now = now_ns();
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    for (const auto& kv : s.svm)
      if (kv.second.dev == dev && !kv.second.in_hbm && kv.second.retry_ns <= now)
        order.emplace_back(kv.second.seq, kv.first);
  }
  if (order.empty()) return 0;
  std::sort(order.begin(), order.end());
  VGPU_REAL_HSA(hsa_agent_get_info);
  uint64_t moved = 0;
  for (const auto& o : order) {
    if (moved >= budget || s.exiting.load()) break;
    std::lock_guard<std::mutex> mg(s.svm_mu);  // a free of this range waits for its migration
    SvmRec rec;
    {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      auto it = s.svm.find(o.second);
      if (it == s.svm.end() || it->second.in_hbm) continue;
      rec = it->second;
    }
    uint64_t avail = 0;
    if (real_hsa_agent_get_info(a.agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MEMORY_AVAIL, &avail) !=
        HSA_STATUS_SUCCESS)
      break;
    const uint64_t avail_raw = avail;
    // ROCr's free-memory figure does not drop as SVM pages move into VRAM (profiles/r4b):
    // what this container and the others on the GPU (node board) hold that way is taken off.
    const uint64_t hidden = hidden_vram(dev);
    avail = avail > hidden ? avail - hidden : 0;
    if (avail < rec.mapped + reserve) break;
    void* p = reinterpret_cast<void*>(o.second);
    int64_t vram0 = -1;
    {
      std::lock_guard<std::mutex> cg(s.ctx_mu);
      // Room under the share (the range counts as resident once moved), decided atomically.
      if (!s.region.promote_spill(s.slot, dev, rec.size, cap)) break;
      s.svm_hbm[dev] += (int64_t)rec.size;
      vram0 = s.hostpid && a.gpu_id ? kfd_vram_usage(s.hostpid, a.gpu_id) : -1;
    }
    const uint64_t t0 = now_ns();
    const Migration m = migrate(p, rec.mapped, a.agent);
    if (m == Migration::kFailed) {
      {
        std::lock_guard<std::mutex> cg(s.ctx_mu);
        s.region.demote_to_spill(s.slot, dev, rec.size);
        s.svm_hbm[dev] -= (int64_t)rec.size;
      }
      // Whatever moved goes back (the failed migration has completed); host memory preferred again.
      if (migrate(p, rec.mapped, a.cpu_agent) == Migration::kPending)
        VLOG_WARN("device %d: moving %p back to host memory is still in progress", dev, p);
      std::lock_guard<std::mutex> g(s.alloc_mu);
      auto it = s.svm.find(o.second);
      if (it != s.svm.end()) it->second.retry_ns = now_ns() + kRetryBackoffNs;
      VLOG_WARN("device %d: %lu spilled bytes at %p could not be promoted into HBM; retrying later", dev,
                (unsigned long)rec.size, p);
      continue;
    }
    if (m == Migration::kPending) {
      // Where the pages end up is the driver's; the range stays charged as HBM data (the
      // conservative side for the other tenants) and is not moved again.
      VLOG_ERROR("device %d: promotion of %lu bytes at %p did not finish within %lu ms; kept as HBM-resident", dev,
                 (unsigned long)rec.size, p, (unsigned long)(migrate_timeout_ns() / 1000000ull));
    }
    if (m == Migration::kDone && rec.mapped >= kBlindProbeBytes && g_avail_blind.load() < 0) {
      // First migration of a size that shows: does ROCr's free figure follow SVM pages?
      const uint64_t after = real_mem_avail(a);
      g_avail_blind.store(avail_raw >= after + rec.mapped / 2 ? 0 : 1);
      VLOG_INFO("device %d: ROCr's free HBM %s SVM pages in VRAM", dev, g_avail_blind.load() ? "omits" : "counts");
    }
    {
      std::lock_guard<std::mutex> cg(s.ctx_mu);
      const int64_t vram1 = vram0 >= 0 && m == Migration::kDone ? kfd_vram_usage(s.hostpid, a.gpu_id) : -1;
      if (s.svm_kfd_vram < 0 && vram0 >= 0 && vram1 >= 0)
        s.svm_kfd_vram = vram1 - vram0 >= (int64_t)rec.mapped / 2 ? 1 : 0;
      s.region.uncharge_host(s.slot, rec.size);
    }
    {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      auto it = s.svm.find(o.second);
      if (it != s.svm.end()) it->second.in_hbm = true;
    }
    moved += rec.size;
    publish_svm_vram();
    VLOG_INFO("device %d: %lu spilled bytes at %p promoted into HBM in %.1f ms", dev, (unsigned long)rec.size, p,
              (now_ns() - t0) / 1e6);
  }
  return moved;
}

// Demotes this process's promoted spills of `dev`, youngest first, until `want` bytes moved:
// back to host memory (the driver migrates the pages: contents intact), charged as spill and
// to the host budget again, and kept there for a back-off. Returns the bytes moved.
uint64_t demote_device(int dev, uint64_t want) {
  ShimState& s = shim();
  AgentInfo& a = s.agents[dev];
  std::vector<std::pair<uint64_t, uintptr_t>> order;  // (seq, ptr) of the promoted spills
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    for (const auto& kv : s.svm)
      if (kv.second.dev == dev && kv.second.in_hbm) order.emplace_back(kv.second.seq, kv.first);
  }
  std::sort(order.rbegin(), order.rend());
  uint64_t moved = 0;
  for (const auto& o : order) {
    if (moved >= want || s.exiting.load()) break;
    std::lock_guard<std::mutex> mg(s.svm_mu);
    SvmRec rec;
    {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      auto it = s.svm.find(o.second);
      if (it == s.svm.end() || !it->second.in_hbm) continue;
      rec = it->second;
    }
    if (s.region.charge_host(s.slot, rec.size) != Charge::kOk) {
      VLOG_WARN("device %d: cannot demote %lu bytes for a co-tenant: the host memory budget is used up", dev,
                (unsigned long)rec.size);
      break;
    }
    void* p = reinterpret_cast<void*>(o.second);
    const uint64_t t0 = now_ns();
    const Migration m = migrate(p, rec.mapped, a.cpu_agent);
    if (m == Migration::kFailed) {
      s.region.uncharge_host(s.slot, rec.size);
      VLOG_WARN("device %d: demotion of %lu bytes at %p failed", dev, (unsigned long)rec.size, p);
      continue;
    }
    {
      std::lock_guard<std::mutex> cg(s.ctx_mu);
      s.region.demote_to_spill(s.slot, dev, rec.size);
      s.svm_hbm[dev] -= (int64_t)rec.size;
    }
    {
      std::lock_guard<std::mutex> g(s.alloc_mu);
      auto it = s.svm.find(o.second);
      if (it != s.svm.end()) {
        it->second.in_hbm = false;
        it->second.retry_ns = now_ns() + kDemoteBackoffNs;
      }
    }
    moved += rec.size;
    publish_svm_vram();
    VLOG_INFO("device %d: %lu promoted bytes at %p demoted to host memory for a co-tenant in %.1f ms", dev,
              (unsigned long)rec.size, p, (now_ns() - t0) / 1e6);
  }
  return moved;
}

// The container was asked to demote `demote_want` bytes of `dev` (its sampler, for a co-tenant
// short of HBM): this process does its part and takes it off the request.
void demote_for_peers(int dev) {
  ShimState& s = shim();
  std::atomic<uint64_t>& want = s.region.raw()->dev[dev].demote_want;
  uint64_t w = want.load(std::memory_order_relaxed);
  if (!w || s.svm_hbm[dev] <= 0) return;
  const uint64_t moved = demote_device(dev, w);
  while (moved && !want.compare_exchange_weak(w, w > moved ? w - moved : 0)) {
  }
}

void* migrator_main(void*) {
  ShimState& s = shim();
  const pid_t me = s.pid;
  const uint64_t period_ns = (uint64_t)std::max(config().util_period_ms, 10) * 1'000'000ull;
  while (!s.exiting.load() && s.pid == me) {
    // Sleeps a period in 5 ms slices, cut short by a free (no condition variable: the shim
    // keeps to glibc 2.17's symbols, test_native_core.py).
    for (uint64_t slept = 0; slept < period_ns && !g_wake.load(std::memory_order_relaxed); slept += 5'000'000) {
      struct timespec ts = {0, 5'000'000};
      nanosleep(&ts, nullptr);
    }
    g_wake.store(false, std::memory_order_relaxed);
    if (s.exiting.load() || !s.active || s.slot < 0) continue;
    for (int d = 0; d < s.n_agents; d++) demote_for_peers(d);
    uint64_t budget = kPromoteBytesPerTick;
    for (int d = 0; d < s.n_agents && budget; d++) budget -= std::min(budget, promote_device(d, budget));
  }
  return nullptr;
}

void start_migrator() {
  bool expected = false;
  if (!config().spill_promote || !g_migrator.compare_exchange_strong(expected, true)) return;
  pthread_t th;
  pthread_attr_t attr;
  pthread_attr_init(&attr);
  pthread_attr_setdetachstate(&attr, PTHREAD_CREATE_DETACHED);
  if (pthread_create(&th, &attr, migrator_main, nullptr) != 0) {
    VLOG_ERROR("cannot start the spill migration thread; spills stay in host memory");
    g_migrator.store(false);
  }
  pthread_attr_destroy(&attr);
}

hsa_status_t pinned_spill(int dev, size_t size, void** ptr) {
  ShimState& s = shim();
  AgentInfo& a = s.agents[dev];
  if (!a.spill_pool.handle) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  VGPU_REAL_HSA(hsa_amd_memory_pool_allocate);
  VGPU_REAL_HSA(hsa_amd_agents_allow_access);
  VGPU_REAL_HSA(hsa_amd_memory_pool_free);
  hsa_status_t st = real_hsa_amd_memory_pool_allocate(a.spill_pool, size, 0, ptr);
  if (st != HSA_STATUS_SUCCESS) return st;
  st = real_hsa_amd_agents_allow_access(1, &a.agent, nullptr, *ptr);
  if (st != HSA_STATUS_SUCCESS) {
    real_hsa_amd_memory_pool_free(*ptr);
    *ptr = nullptr;
  }
  return st;
}

}  // namespace

// Spilled bytes are host memory the container holds: they count against its host budget
// (VGPU_HOST_MEMORY_LIMIT, shared with hipHostMalloc / hipHostRegister), so the RAM an
// oversubscribed vGPU takes is bounded like any other (plugin/host_memory.py sizes the
// budget and refuses scalings the node cannot back). The caller has charged `size` as data.
hsa_status_t spill_allocate(int dev, size_t size, void** ptr) {
  ShimState& s = shim();
  const Config& cfg = config();
  if (s.region.charge_host(s.slot, size) != Charge::kOk) {
    VLOG_WARN("device %d: %zu bytes cannot spill: host memory budget %lu (in use %lu) is used up", dev, size,
              (unsigned long)s.region.host_limit(), (unsigned long)s.region.host_usage());
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  }
  hsa_status_t st = HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  // svm (default): an SVM range, promotable into HBM later; pinned host memory only where the
  // driver has no SVM. auto: below VGPU_SPILL_LARGE pinned host memory (never moves), large
  // ones SVM ranges. Neither placement exports over IPC on MI355X - KFD shares device memory
  // only (tests/test_gpu_spill_ipc.py, profiles/r5e).
  const bool small = cfg.spill_backing == SpillBacking::kAuto && size < cfg.spill_large_bytes;
  const bool want_svm = cfg.spill_backing != SpillBacking::kPinned && !small && s.agents[dev].cpu_agent.handle;
  const bool svm_ok = want_svm && svm_supported();
  if (svm_ok) {
    size_t mapped = 0;
    st = svm_map(dev, size, ptr, &mapped);
    if (st == HSA_STATUS_SUCCESS) {
      s.region.uncharge(s.slot, dev, size, kMemData);
      s.region.force_charge(s.slot, dev, size, kMemSpill);
      {
        std::lock_guard<std::mutex> g(s.alloc_mu);
        s.svm[reinterpret_cast<uintptr_t>(*ptr)] = SvmRec{size, mapped, dev, false, g_seq.fetch_add(1), 0};
      }
      VLOG_INFO("device %d: %zu bytes spilled to host memory at %p (SVM, promotable)", dev, size, *ptr);
      start_migrator();
      return st;
    }
    VLOG_WARN("device %d: SVM spill of %zu bytes refused (status %d)%s", dev, size, (int)st,
              cfg.spill_backing == SpillBacking::kSvm ? "" : "; using pinned host memory");
  }
  if (cfg.spill_backing != SpillBacking::kSvm || !svm_ok) st = pinned_spill(dev, size, ptr);
  if (st != HSA_STATUS_SUCCESS && small && s.agents[dev].cpu_agent.handle && svm_supported()) {
    size_t mapped = 0;  // no pinned memory left for a small one: an SVM range still serves it
    st = svm_map(dev, size, ptr, &mapped);
    if (st == HSA_STATUS_SUCCESS) {
      s.region.uncharge(s.slot, dev, size, kMemData);
      s.region.force_charge(s.slot, dev, size, kMemSpill);
      {
        std::lock_guard<std::mutex> g(s.alloc_mu);
        s.svm[reinterpret_cast<uintptr_t>(*ptr)] = SvmRec{size, mapped, dev, false, g_seq.fetch_add(1), 0};
      }
      start_migrator();
      return st;
    }
  }
  if (st != HSA_STATUS_SUCCESS) {
    s.region.uncharge_host(s.slot, size);
    return st;
  }
  s.region.uncharge(s.slot, dev, size, kMemData);
  s.region.force_charge(s.slot, dev, size, kMemSpill);
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    s.allocs[reinterpret_cast<uintptr_t>(*ptr)] = AllocRec{size, dev, kMemSpill};
  }
  VLOG_INFO("device %d: %zu bytes spilled to pinned host memory at %p", dev, size, *ptr);
  return HSA_STATUS_SUCCESS;
}

bool spill_release(void* ptr) {
  ShimState& s = shim();
  if (!ptr) return false;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    if (!s.svm.count(reinterpret_cast<uintptr_t>(ptr))) return false;
  }
  std::lock_guard<std::mutex> mg(s.svm_mu);  // not while the range migrates
  SvmRec rec;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    auto it = s.svm.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == s.svm.end()) return true;  // freed concurrently
    rec = it->second;
    s.svm.erase(it);
  }
  if (s.slot >= 0 && !s.exiting.load()) {
    if (rec.in_hbm) {
      std::lock_guard<std::mutex> cg(s.ctx_mu);
      s.region.uncharge(s.slot, rec.dev, rec.size, kMemData);
      s.svm_hbm[rec.dev] -= (int64_t)rec.size;
    } else {
      s.region.uncharge(s.slot, rec.dev, rec.size, kMemSpill);
      s.region.uncharge_host(s.slot, rec.size);
    }
  }
  munmap(ptr, rec.mapped);  // KFD drops the range (and its VRAM) with the mapping
  return true;
}

void notify_device_memory_freed() {
  if (g_migrator.load(std::memory_order_relaxed)) g_wake.store(true, std::memory_order_relaxed);
}

bool svm_allow_access(const void* ptr, uint32_t n, const hsa_agent_t* agents, hsa_status_t* st) {
  ShimState& s = shim();
  size_t mapped = 0;
  {
    std::lock_guard<std::mutex> g(s.alloc_mu);
    auto it = s.svm.find(reinterpret_cast<uintptr_t>(ptr));
    if (it == s.svm.end()) return false;
    mapped = it->second.mapped;
  }
  VGPU_REAL_HSA(hsa_amd_svm_attributes_set);
  std::vector<hsa_amd_svm_attribute_pair_t> attrs;
  for (uint32_t i = 0; i < n; i++) attrs.push_back({HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE, agents[i].handle});
  *st = attrs.empty() ? HSA_STATUS_SUCCESS
                      : real_hsa_amd_svm_attributes_set(const_cast<void*>(ptr), mapped, attrs.data(), attrs.size());
  return true;
}

int64_t svm_hbm_outside_kfd(int dev) {
  ShimState& s = shim();
  return s.svm_kfd_vram == 1 ? 0 : s.svm_hbm[dev];
}

uint64_t hidden_vram(int dev) {
  ShimState& s = shim();
  if (dev < 0 || dev >= s.n_agents || !s.region.attached() || g_avail_blind.load(std::memory_order_relaxed) == 0)
    return 0;
  const Region* r = s.region.raw();
  // The container's sum, with this process's current bytes for what it last published.
  const uint64_t mine_pub = s.slot >= 0 ? r->procs[s.slot].used[dev].svm_vram.load(std::memory_order_relaxed) : 0;
  const uint64_t container = s.region.svm_vram(dev);
  const uint64_t own = (container > mine_pub ? container - mine_pub : 0) + own_svm_vram(s, dev);
  return own + r->dev[dev].node_svm_vram.load(std::memory_order_relaxed);
}

void publish_svm_vram() {
  ShimState& s = shim();
  if (s.slot < 0 || !s.region.attached()) return;
  for (int d = 0; d < s.n_agents; d++) s.region.set_svm_vram(s.slot, d, own_svm_vram(s, d));
}

hsa_status_t reclaim_peer_hbm(int dev, size_t size, hsa_status_t (*attempt)(void*), void* ctx) {
  ShimState& s = shim();
  const Config& cfg = config();
  Region* r = s.region.raw();
  if (cfg.demote_wait_ms <= 0 || dev < 0 || dev >= s.n_agents || !r->dev[dev].node_svm_vram.load())
    return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  DeviceState& d = r->dev[dev];
  VLOG_INFO("device %d: %zu bytes refused by the driver within the quota; co-tenants hold %lu bytes of promoted "
            "spills here - asking them to demote", dev, size, (unsigned long)d.node_svm_vram.load());
  const uint64_t t0 = now_ns(), limit = (uint64_t)cfg.demote_wait_ms * 1'000'000ull;
  uint64_t asked = 0;
  hsa_status_t st = HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  trace_push("vgpu:reclaim");
  for (uint64_t el = 0; el < limit; el = now_ns() - t0) {
    if (!asked || el - asked >= 1'000'000'000ull) {  // (re-)published every second: a fresh request
      d.hbm_want.store(std::max<uint64_t>(size, d.hbm_want.load()));
      d.hbm_want_ns.store(now_ns());
      asked = std::max<uint64_t>(el, 1);
    }
    struct timespec ts = {0, 20'000'000};
    nanosleep(&ts, nullptr);
    st = attempt(ctx);
    if (st != HSA_STATUS_ERROR_OUT_OF_RESOURCES) break;
  }
  d.hbm_want_ns.store(0);
  d.hbm_want.store(0);
  trace_pop();
  VLOG_INFO("device %d: %zu bytes %s after %.0f ms", dev, size, st == HSA_STATUS_SUCCESS ? "allocated" : "still refused",
            (now_ns() - t0) / 1e6);
  return st;
}

void svm_recharge(int slot, uint64_t* host) {
  ShimState& s = shim();
  for (const auto& kv : s.svm) {
    if (kv.second.in_hbm) {
      s.region.force_charge(slot, kv.second.dev, kv.second.size, kMemData);
    } else {
      s.region.force_charge(slot, kv.second.dev, kv.second.size, kMemSpill);
      *host += kv.second.size;
    }
  }
}

void svm_forget() {
  ShimState& s = shim();
  s.svm.clear();
  for (auto& b : s.svm_hbm) b = 0;
  new (&s.svm_mu) std::mutex();
  g_migrator.store(false);
  g_wake.store(false);
}

}  // namespace vgpu
