// The tenant's own shared virtual memory: device memory placed through SVM attributes is
// held to the device quota like any other.
//
// KFD's SVM API registers an ordinary range of a process's memory for GPU access and moves
// it into a GPU's HBM on request (hsa_amd_svm_prefetch_async) or, with recoverable page
// faults, towards its preferred location (HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION). Neither
// passes an allocation entry point, and ROCr's free-memory figure does not show migrated
// pages (profiles/r4b); KFD's per-process vram_<gpu_id> does (profiles/r5b), so the OOM killer
// would catch a large escape after the fact - these hooks refuse it before the driver sees it. libamdhip64 imports both entry points: hipMemAdvise and hipMemPrefetchAsync on
// system-allocated memory reach them as well.
//
// Reference: cuMemAllocManaged is an accounted allocation ([memory.c:216-223], oom_check +
// add_chunk_only); UVM migrations after that are the driver's, within the charged size.
// Here the unit is the range, as SVM has no allocation: a range (page-granular) that gets a
// GPU as prefetch target - or as preferred location where XNACK lets pages migrate on fault
// - is admitted against that device's quota (CAS admission, HSA_STATUS_ERROR_OUT_OF_RESOURCES
// past it, before the runtime sees the call); a range prefetched back to the CPU (and, with
// XNACK, its preferred location cleared) gives its charge back; a range the process unmapped is dropped by the maintenance thread
// (svm_tenant_reconcile, from /proc/self/maps). Excluded: the shim's own spills (spill.cpp,
// charged as spill / promoted data) and memory charged at allocation (pool allocations,
// hipMallocManaged - whose own SVM calls pass while it runs).
#include <sys/mman.h>
#include <unistd.h>

#include <algorithm>
#include <cstdio>
#include <mutex>
#include <utility>
#include <vector>

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"

namespace vgpu {

thread_local bool t_managed_alloc = false;

namespace {

using Interval = std::pair<uintptr_t, uintptr_t>;  // [first, second)

uintptr_t page_down(uintptr_t a) { return a & ~((uintptr_t)sysconf(_SC_PAGESIZE) - 1); }
uintptr_t page_up(uintptr_t a) {
  const uintptr_t pg = (uintptr_t)sysconf(_SC_PAGESIZE);
  return (a + pg - 1) & ~(pg - 1);
}

// Device ordinal of an agent as a placement: a GPU of this process, or -1 (a CPU agent, the
// null agent, anything else).
int placement(uint64_t agent_handle) {
  if (!agent_handle) return -1;
  return agent_ordinal(hsa_agent_t{agent_handle});
}

// Ranges inside [a, b) charged elsewhere: the shim's SVM spills and recorded allocations.
std::vector<Interval> exempt_within(uintptr_t a, uintptr_t b) {
  ShimState& s = shim();
  std::vector<Interval> out;
  std::lock_guard<std::mutex> g(s.alloc_mu);
  auto add = [&](uintptr_t p, uint64_t len) {
    const uintptr_t lo = std::max(a, page_down(p)), hi = std::min(b, page_up(p + len));
    if (lo < hi) out.emplace_back(lo, hi);
  };
  for (const auto& kv : s.svm) add(kv.first, kv.second.mapped);
  for (const auto& kv : s.managed) add(kv.first, kv.second.size);
  for (const auto& kv : s.allocs) add(kv.first, kv.second.size);
  std::sort(out.begin(), out.end());
  return out;
}

// [a, b) less the exempt intervals.
std::vector<Interval> subtract(uintptr_t a, uintptr_t b, const std::vector<Interval>& ex) {
  std::vector<Interval> out;
  uintptr_t cur = a;
  for (const Interval& e : ex) {
    if (e.second <= cur) continue;
    if (e.first >= b) break;
    if (e.first > cur) out.emplace_back(cur, e.first);
    cur = std::max(cur, e.second);
  }
  if (cur < b) out.emplace_back(cur, b);
  return out;
}

// Splits the segment that strictly contains `at` (tsvm_mu held).
void split_at(std::map<uintptr_t, TenantSvmSeg>& m, uintptr_t at) {
  auto it = m.upper_bound(at);
  if (it == m.begin()) return;
  --it;
  if (it->first < at && it->second.end > at) {
    TenantSvmSeg tail = it->second;
    it->second.end = at;
    m.emplace(at, tail);
  }
}

// Recoverable GPU page faults (XNACK): only then do pages move towards their preferred
// location by themselves; without them a range is in VRAM only where it was prefetched.
bool xnack_on() {
  static const bool on = [] {
    VGPU_REAL_HSA(hsa_system_get_info);
    bool x = false;
    return real_hsa_system_get_info &&
           real_hsa_system_get_info((hsa_system_info_t)HSA_AMD_SYSTEM_INFO_XNACK_ENABLED, &x) == HSA_STATUS_SUCCESS &&
           x;
  }();
  return on;
}

int charged_dev(const TenantSvmSeg& g) { return g.loc >= 0 ? g.loc : xnack_on() ? g.pref : -1; }

// Moves `bytes` of charge bookkeeping for device `dev` (ctx_mu held): +1 adds, -1 removes.
void count(int dev, bool in_vram, int sign, uint64_t bytes) {
  ShimState& s = shim();
  if (dev < 0) return;
  (in_vram ? s.tsvm_loc : s.tsvm_pref)[dev] += sign * (int64_t)bytes;
}

enum class Field { kPref, kLoc };

// Applies a placement change to [a, b) of the tenant's ranges: admits the bytes that become
// charged on a device, calls the runtime, then commits (or undoes everything if the runtime
// refused). Returns the runtime's status, or OUT_OF_RESOURCES past the quota.
template <typename Call>
hsa_status_t place(uintptr_t a, uintptr_t b, Field field, int dev, Call call) {
  ShimState& s = shim();
  if (dev >= 0 && !s.agents[dev].authorised) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  std::lock_guard<std::mutex> tg(s.tsvm_mu);
  auto& m = s.tsvm;
  // The pieces of the range this call decides about, as (start, end, old segment) - a gap
  // in the map is a fresh range (host memory, no preference).
  struct Piece {
    uintptr_t lo, hi;
    TenantSvmSeg before, after;
  };
  std::vector<Piece> pieces;
  for (const Interval& iv : subtract(a, b, exempt_within(a, b))) {
    split_at(m, iv.first);
    split_at(m, iv.second);
    uintptr_t cur = iv.first;
    auto it = m.lower_bound(iv.first);
    while (cur < iv.second) {
      TenantSvmSeg before{0, -1, -1, -1};
      uintptr_t hi;
      if (it != m.end() && it->first == cur) {
        before = it->second;
        hi = std::min(it->second.end, iv.second);
        ++it;
      } else {
        hi = it != m.end() && it->first < iv.second ? it->first : iv.second;
      }
      TenantSvmSeg after = before;
      after.end = hi;
      (field == Field::kPref ? after.pref : after.loc) = dev;
      after.charged = charged_dev(after);
      pieces.push_back(Piece{cur, hi, before, after});
      cur = hi;
    }
  }
  // Admission: the bytes each device gains (a device the range leaves is uncharged only
  // once the runtime has moved it).
  uint64_t gain[kMaxDevices] = {};
  for (const Piece& p : pieces)
    if (p.after.charged >= 0 && p.after.charged != p.before.charged) gain[p.after.charged] += p.hi - p.lo;
  for (int d = 0; d < s.n_agents; d++) {
    if (!gain[d]) continue;
    if (s.region.charge(s.slot, d, gain[d], kMemData) != Charge::kOk) {
      VLOG_WARN("device %d OOM (SVM range %#lx+%lu): usage %lu of limit %lu", d, (unsigned long)a,
                (unsigned long)(b - a), (unsigned long)s.region.usage(d), (unsigned long)s.region.limit(d));
      for (int u = 0; u < d; u++)
        if (gain[u]) s.region.uncharge(s.slot, u, gain[u], kMemData);
      return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
    }
  }
  const hsa_status_t st = call();
  std::lock_guard<std::mutex> cg(s.ctx_mu);  // context resync reads the counts
  if (st != HSA_STATUS_SUCCESS) {
    for (int d = 0; d < s.n_agents; d++)
      if (gain[d]) s.region.uncharge(s.slot, d, gain[d], kMemData);
    return st;
  }
  for (const Piece& p : pieces) {
    const uint64_t len = p.hi - p.lo;
    count(p.before.charged, p.before.loc >= 0, -1, len);
    count(p.after.charged, p.after.loc >= 0, +1, len);
    if (p.before.charged >= 0 && p.before.charged != p.after.charged)
      s.region.uncharge(s.slot, p.before.charged, len, kMemData);
    if (p.after.pref < 0 && p.after.loc < 0) m.erase(p.lo);  // host memory, no preference: forgotten
    else m[p.lo] = p.after;
  }
  VLOG_DEBUG("SVM range %#lx+%lu: %s -> device %d", (unsigned long)a, (unsigned long)(b - a),
             field == Field::kPref ? "preferred location" : "prefetch", dev);
  return st;
}

bool tracking() {
  ShimState& s = shim();
  if (__builtin_expect(s.phase.load(std::memory_order_acquire) == 0, 0)) shim_init_after_hsa();
  return s.phase.load(std::memory_order_acquire) == 2 && s.active && s.slot >= 0 && !s.exiting.load() &&
         !t_managed_alloc;
}

}  // namespace

int64_t svm_tenant_outside_kfd(int dev) {
  ShimState& s = shim();
  if (dev < 0 || dev >= kMaxDevices) return 0;
  // Pages only preferred on a device never left host memory; prefetched ones are in VRAM,
  // which KFD's per-process counter shows (measured on MI355X, profiles/r5b) unless a spill
  // promotion found otherwise (spill.cpp measures it around its first migration).
  return s.tsvm_pref[dev] + (s.svm_kfd_vram == 0 ? s.tsvm_loc[dev] : 0);
}

void svm_tenant_reconcile() {
  ShimState& s = shim();
  {
    std::lock_guard<std::mutex> tg(s.tsvm_mu);
    if (s.tsvm.empty()) return;
  }
  // The process's mappings: KFD drops an SVM range (and its VRAM) when it is unmapped.
  std::vector<Interval> maps;
  if (FILE* f = fopen("/proc/self/maps", "r")) {
    char line[512];
    while (fgets(line, sizeof(line), f)) {
      unsigned long lo = 0, hi = 0;
      if (sscanf(line, "%lx-%lx", &lo, &hi) == 2 && lo < hi) {
        if (!maps.empty() && maps.back().second == lo) maps.back().second = hi;
        else maps.emplace_back(lo, hi);
      }
    }
    fclose(f);
  } else {
    return;
  }
  std::lock_guard<std::mutex> tg(s.tsvm_mu);
  std::lock_guard<std::mutex> cg(s.ctx_mu);
  std::map<uintptr_t, TenantSvmSeg> kept;
  for (const auto& kv : s.tsvm) {
    const uintptr_t a = kv.first, b = kv.second.end;
    uint64_t mapped = 0;
    auto it = std::upper_bound(maps.begin(), maps.end(), Interval{a, ~(uintptr_t)0});
    if (it != maps.begin()) --it;
    for (; it != maps.end() && it->first < b; ++it) {
      const uintptr_t lo = std::max(a, it->first), hi = std::min(b, it->second);
      if (lo >= hi) continue;
      TenantSvmSeg g = kv.second;
      g.end = hi;
      kept[lo] = g;
      mapped += hi - lo;
    }
    const uint64_t gone = (b - a) - mapped;
    if (!gone) continue;
    count(kv.second.charged, kv.second.loc >= 0, -1, gone);
    if (kv.second.charged >= 0) s.region.uncharge(s.slot, kv.second.charged, gone, kMemData);
    VLOG_DEBUG("SVM range %#lx+%lu: %lu bytes unmapped, charge released", (unsigned long)a, (unsigned long)(b - a),
               (unsigned long)gone);
  }
  s.tsvm.swap(kept);
}

void svm_tenant_recharge(int slot) {
  ShimState& s = shim();
  std::lock_guard<std::mutex> tg(s.tsvm_mu);
  for (const auto& kv : s.tsvm)
    if (kv.second.charged >= 0) s.region.force_charge(slot, kv.second.charged, kv.second.end - kv.first, kMemData);
}

void svm_tenant_forget() {
  ShimState& s = shim();
  new (&s.tsvm_mu) std::mutex();  // may be held by a parent thread that does not exist here
  s.tsvm.clear();
  for (auto& b : s.tsvm_loc) b = 0;
  for (auto& b : s.tsvm_pref) b = 0;
}

}  // namespace vgpu

using namespace vgpu;

extern "C" {

hsa_status_t hsa_amd_svm_attributes_set(void* ptr, size_t size, hsa_amd_svm_attribute_pair_t* attribute_list,
                                        size_t attribute_count) {
  VGPU_REAL_HSA(hsa_amd_svm_attributes_set);
  if (!real_hsa_amd_svm_attributes_set) return HSA_STATUS_ERROR;
  auto real = [&] { return real_hsa_amd_svm_attributes_set(ptr, size, attribute_list, attribute_count); };
  if (!ptr || !size || !attribute_list || !tracking()) return real();
  // The last preferred-location entry of the list decides (the runtime applies them in order).
  int pref = -2;
  for (size_t i = 0; i < attribute_count; i++)
    if (attribute_list[i].attribute == HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION) pref = placement(attribute_list[i].value);
  if (pref == -2) return real();
  gate_suspend();
  const uintptr_t a = page_down(reinterpret_cast<uintptr_t>(ptr)), b = page_up(reinterpret_cast<uintptr_t>(ptr) + size);
  return place(a, b, Field::kPref, pref, real);
}

hsa_status_t hsa_amd_svm_prefetch_async(void* ptr, size_t size, hsa_agent_t agent, uint32_t num_dep_signals,
                                        const hsa_signal_t* dep_signals, hsa_signal_t completion_signal) {
  VGPU_REAL_HSA(hsa_amd_svm_prefetch_async);
  if (!real_hsa_amd_svm_prefetch_async) return HSA_STATUS_ERROR;
  auto real = [&] {
    return real_hsa_amd_svm_prefetch_async(ptr, size, agent, num_dep_signals, dep_signals, completion_signal);
  };
  if (!ptr || !size || !tracking()) return real();
  gate_suspend();
  const uintptr_t a = page_down(reinterpret_cast<uintptr_t>(ptr)), b = page_up(reinterpret_cast<uintptr_t>(ptr) + size);
  return place(a, b, Field::kLoc, placement(agent.handle), real);
}

}  // extern "C"
