#include "vgpu/region_api.h"

#include <cerrno>
#include <cstring>
#include <new>

#include "vgpu/cumask.h"
#include "vgpu/region.h"

using namespace vgpu;

struct vgpu_region {
  SharedRegion r;
};

extern "C" {

vgpu_region* vgpu_region_open(const char* path, int create, int* err) {
  vgpu_region* h = new (std::nothrow) vgpu_region();
  if (!h) {
    if (err) *err = -ENOMEM;
    return nullptr;
  }
  int rc = h->r.attach(path, nullptr, create != 0);
  if (err) *err = rc;
  if (rc != 0) {
    delete h;
    return nullptr;
  }
  return h;
}

void vgpu_region_close(vgpu_region* r) { delete r; }
uint32_t vgpu_region_version(void) { return kRegionVersion; }
uint64_t vgpu_region_size(void) { return sizeof(Region); }
int vgpu_region_num_devices(vgpu_region* r) { return r->r.num_devices(); }

int vgpu_region_device_info(vgpu_region* r, int dev, vgpu_device_info* out) {
  if (dev < 0 || dev >= kMaxDevices) return -EINVAL;
  const DeviceState& d = r->r.raw()->dev[dev];
  memset(out, 0, sizeof(*out));
  memcpy(out->uuid, d.uuid, sizeof(out->uuid));
  out->mem_limit = d.mem_limit;
  out->phys_total = d.phys_total;
  out->used = d.used.load();
  out->spilled = d.spilled.load();
  out->monitor_used = d.monitor_used.load();
  out->cu_limit_pct = d.cu_limit_pct;
  out->cu_count = d.cu_count;
  out->num_xcc = d.num_xcc;
  CuMask m;
  memcpy(m.words, d.cu_mask, sizeof(m.words));
  m.nbits = d.cu_mask_bits;
  out->cu_mask_count = m.count();
  memcpy(out->cu_mask, d.cu_mask, sizeof(out->cu_mask));
  out->credit_ns = d.credit_ns.load();
  out->charged_ns = d.charged_ns.load();
  out->wall_ns = d.wall_ns.load();
  out->util_pct = (d.util_pm.load() + 5) / 10;
  out->cu_mode = d.cu_mode.load();
  out->gpu_id = d.gpu_id;
  out->bdf = d.bdf;
  out->domain = d.domain;
  out->configured = d.configured;
  out->hbm_limit = d.hbm_limit;
  out->crowd = d.crowd.load();
  out->preempt = d.preempt.load();
  out->depth_cap = d.depth_cap.load();
  out->cu_share_bp = d.cu_share_bp;
  return 0;
}

int vgpu_region_proc_count(vgpu_region* r) { return r->r.raw()->hdr.proc_num.load(); }

int vgpu_region_procs(vgpu_region* r, vgpu_proc_info* out, int max) {
  int n = 0;
  const Region* g = r->r.raw();
  for (int i = 0; i < kMaxProcs && n < max; i++) {
    const ProcSlot& s = g->procs[i];
    if (!s.pid.load()) continue;
    vgpu_proc_info& o = out[n++];
    memset(&o, 0, sizeof(o));
    o.pid = s.pid.load();
    o.hostpid = s.hostpid.load();
    o.status = s.status.load();
    o.priority = s.priority;
    o.launches = s.launches.load();
    o.throttle_ns = s.throttle_ns.load();
    o.suspend_ns = s.suspend_ns.load();
    o.oom_events = s.oom_events.load();
    for (int d = 0; d < kMaxDevices; d++) {
      o.used[d] = s.used[d].total.load();
      o.peak[d] = s.used[d].peak.load();
      for (int k = 0; k < kMemKinds; k++) o.used_kind[d][k] = s.used[d].kind[k].load();
    }
    o.host_used = s.host_used.load();
    o.host_peak = s.host_peak.load();
  }
  return n;
}

int vgpu_region_set_memory_limit(vgpu_region* r, int dev, uint64_t bytes) {
  if (dev < 0 || dev >= kMaxDevices) return -EINVAL;
  r->r.set_limit(dev, bytes);
  return 0;
}

int vgpu_region_set_cu_limit(vgpu_region* r, int dev, int pct) {
  if (dev < 0 || dev >= kMaxDevices || pct < 0 || pct > 100) return -EINVAL;
  r->r.set_cu_limit(dev, pct);
  return 0;
}

int vgpu_region_set_cu_share(vgpu_region* r, int dev, int bp) {
  if (dev < 0 || dev >= kMaxDevices || bp < 0 || bp > 10000) return -EINVAL;
  r->r.raw()->dev[dev].cu_share_bp = bp;
  r->r.raw()->hdr.generation.fetch_add(1);
  return 0;
}

int vgpu_region_set_hbm_limit(vgpu_region* r, int dev, uint64_t bytes) {
  if (dev < 0 || dev >= kMaxDevices) return -EINVAL;
  r->r.raw()->dev[dev].hbm_limit = bytes;
  r->r.raw()->hdr.generation.fetch_add(1);
  return 0;
}

int vgpu_region_suspend_all(vgpu_region* r) {
  r->r.suspend_all();
  return 0;
}
int vgpu_region_resume_all(vgpu_region* r) {
  r->r.resume_all();
  return 0;
}
int vgpu_region_suspended(vgpu_region* r) { return r->r.raw()->hdr.suspend_all.load(); }
int vgpu_region_set_priority(vgpu_region* r, int prio) {
  r->r.raw()->hdr.priority.store(prio);
  return 0;
}
int vgpu_region_get_priority(vgpu_region* r) { return r->r.raw()->hdr.priority.load(); }
int vgpu_region_set_recent_kernel(vgpu_region* r, int v) {
  r->r.raw()->hdr.recent_kernel.store(v);
  return 0;
}
int vgpu_region_get_recent_kernel(vgpu_region* r) { return r->r.raw()->hdr.recent_kernel.load(); }

uint64_t vgpu_region_samples(vgpu_region* r) { return r->r.raw()->hdr.samples.load(); }

uint64_t vgpu_region_other_refreshes(vgpu_region* r) { return r->r.raw()->hdr.other_refreshes.load(); }
int vgpu_region_set_utilization_switch(vgpu_region* r, int v) {
  r->r.raw()->hdr.utilization_switch.store(v);
  return 0;
}
int vgpu_region_reclaim(vgpu_region* r) { return r->r.reclaim_dead(); }

int vgpu_region_host_info(vgpu_region* r, uint64_t* limit, uint64_t* used) {
  if (limit) *limit = r->r.host_limit();
  if (used) *used = r->r.host_usage();
  return 0;
}

int vgpu_region_set_host_limit(vgpu_region* r, uint64_t bytes) {
  r->r.set_host_limit(bytes);
  return 0;
}

int vgpu_region_charge_host(vgpu_region* r, int slot, uint64_t bytes) {
  return r->r.charge_host(slot, bytes) == Charge::kOk ? 0 : -ENOMEM;
}

void vgpu_region_uncharge_host(vgpu_region* r, int slot, uint64_t bytes) { r->r.uncharge_host(slot, bytes); }
int vgpu_region_register(vgpu_region* r, int32_t pid, int32_t hostpid) {
  return r->r.register_process(pid, hostpid, 1);
}
void vgpu_region_unregister(vgpu_region* r, int slot) { r->r.unregister_process(slot); }
int vgpu_region_charge(vgpu_region* r, int slot, int dev, uint64_t bytes, int kind) {
  if (dev < 0 || dev >= kMaxDevices || kind < 0 || kind >= kMemKinds) return -EINVAL;
  return r->r.charge(slot, dev, bytes, (MemKind)kind) == Charge::kOk ? 0 : 1;
}
void vgpu_region_uncharge(vgpu_region* r, int slot, int dev, uint64_t bytes, int kind) {
  if (dev < 0 || dev >= kMaxDevices || kind < 0 || kind >= kMemKinds) return;
  r->r.uncharge(slot, dev, bytes, (MemKind)kind);
}
int vgpu_cu_share_count(int cu_count, int num_xcc, int pct) { return cu_share_count(cu_count, num_xcc, pct); }
void vgpu_cu_partition_range(int cu_count, int num_xcc, int split, int slot, int* begin, int* end) {
  cu_partition_range(cu_count, num_xcc, split, slot, begin, end);
}
int64_t vgpu_parse_size(const char* s) {
  uint64_t v = 0;
  return parse_size(s, &v) ? (int64_t)v : -1;
}

}  // extern "C"
