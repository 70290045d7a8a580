// amd-smi / rocm-smi virtualisation: in-container tools see the container's GPUs, its
// processes and the vGPU quota.
//
// Reference: src/nvml/hook.c nvmlDeviceGetMemoryInfo(_v2) [327-361] reports
// total = limit, used = region usage (or the monitor value under MEMORY_OVERRIDE),
// free = limit - used; nvmlDeviceGetCount / GetHandleByIndex / ByPciBusId / ByUUID
// [438-527] remap the device list to the container's virtual devices.
//
// MI355X equivalents:
//  * memory: amdsmi_get_gpu_memory_total/usage, amdsmi_get_gpu_vram_usage and the
//    rocm_smi rsmi_dev_memory_total/usage_get calls;
//  * devices: amdsmi is handle based, so filtering amdsmi_get_processor_handles to the
//    container's GPUs (the plugin's VGPU_DEVICE_BDFS, else the BDFs the container's GPU
//    processes recorded in the region) virtualises every later per-device query without
//    per-function index remapping. rocm_smi is index based: rsmi_num_monitor_devices
//    reports the container's GPUs and every index-taking entry point (97 of them,
//    generated from the header into rsmi_remap_gen.inc) translates the container's
//    index into the node's; rsmi_compute_process_gpus_get maps back;
//  * processes: amdsmi_get_gpu_process_list and rsmi_compute_process_info(_by_pid)_get
//    keep only the container's processes (the region's host PIDs), so tenants cannot see
//    each other's workloads.
// These run in processes that usually never initialise ROCr (amd-smi itself), so the
// region is attached read-mostly and devices are matched by PCI BDF.
#include <amd_smi/amdsmi.h>
#include <rocm_smi/rocm_smi.h>

#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <vector>

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"

using namespace vgpu;

namespace {

constexpr uint64_t kNoGpuId = ~0ull;

// Region device index for a PCI (domain, bdfid) pair, or -1. Compute partitions exposed
// as GPUs share one PCI address: then the KFD gpu_id (`gpu_id`, kNoGpuId when the SMI
// library cannot tell) picks the device.
int device_by_bdf(uint64_t domain, uint32_t bdfid, uint64_t gpu_id = kNoGpuId) {
  if (!shim_attach_region_only()) return -1;
  if (!config().hook_smi) return -1;
  const Region* r = shim().region.raw();
  int first = -1, unknown = -1;
  for (int i = 0; i < kMaxDevices; i++) {
    const DeviceState& d = r->dev[i];
    if (!d.configured || d.bdf != bdfid || d.domain != (uint32_t)domain) continue;
    if (gpu_id != kNoGpuId && d.gpu_id == (uint32_t)gpu_id) return i;
    if (first < 0) first = i;
    if (unknown < 0 && !d.gpu_id) unknown = i;
  }
  // A partition at this address that is not one of the region's devices is another
  // container's: no virtualisation for it (unless the region does not know gpu_ids).
  return gpu_id == kNoGpuId ? first : unknown;
}

// KFD gpu_id of an amd-smi processor (kNoGpuId when unsupported).
uint64_t amdsmi_gpu_id(amdsmi_processor_handle h) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_kfd_info, "libamd_smi", nullptr);
  amdsmi_kfd_info_t k;
  memset(&k, 0, sizeof(k));
  if (!real_amdsmi_get_gpu_kfd_info || real_amdsmi_get_gpu_kfd_info(h, &k) != AMDSMI_STATUS_SUCCESS) return kNoGpuId;
  return k.kfd_id == 0xFFFFFFFFFFFFFFFFull ? kNoGpuId : k.kfd_id;
}

uint64_t virt_total(int dev, uint64_t real_total) {
  uint64_t lim = shim().region.limit(dev);
  if (!lim) return real_total;
  return (config().oversubscribe || lim < real_total) ? lim : real_total;
}

uint64_t virt_used(int dev) {
  const Region* r = shim().region.raw();
  if (config().memory_override) return r->dev[dev].monitor_used.load();
  return r->dev[dev].used.load();
}

// Whether several of the region's devices sit at PCI address `b` (compute partitions).
bool shared_bdf(amdsmi_bdf_t b) {
  if (!shim_attach_region_only()) return false;
  const Region* r = shim().region.raw();
  int n = 0;
  for (int i = 0; i < kMaxDevices; i++) {
    const DeviceState& d = r->dev[i];
    n += d.configured && d.bdf == (uint32_t)(b.as_uint & 0xffff) && d.domain == (uint32_t)(b.as_uint >> 16);
  }
  return n > 1;
}

int amdsmi_dev(amdsmi_processor_handle h) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_device_bdf, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_device_bdf) return -1;
  amdsmi_bdf_t b;
  b.as_uint = 0;
  if (real_amdsmi_get_gpu_device_bdf(h, &b) != AMDSMI_STATUS_SUCCESS) return -1;
  return device_by_bdf(b.as_uint >> 16, (uint32_t)(b.as_uint & 0xffff), shared_bdf(b) ? amdsmi_gpu_id(h) : kNoGpuId);
}

// The container's GPUs as (domain, bdfid) pairs: VGPU_DEVICE_BDFS from the plugin
// ("dddd:bb:dd.f,..."), else the region's recorded devices. Empty = no filtering.
struct Bdf {
  uint64_t domain;
  uint32_t bdfid;
  uint64_t gpu_id = kNoGpuId;  // KFD gpu_id when known (partitions share an address)
};

std::vector<Bdf> visible_bdfs() {
  std::vector<Bdf> out;
  const bool attached = shim_attach_region_only();  // also loads the env config
  if (!config().hook_smi || config().disabled) return out;
  if (const char* s = getenv("VGPU_DEVICE_BDFS")) {
    const char* p = s;
    while (*p) {
      unsigned dom = 0, bus = 0, dev = 0, fn = 0;
      int used = 0;
      if (sscanf(p, "%x:%x:%x.%x%n", &dom, &bus, &dev, &fn, &used) == 4) {
        out.push_back({dom, (bus << 8) | (dev << 3) | fn});
        p += used;
      } else {
        VLOG_WARN("invalid VGPU_DEVICE_BDFS=%s: device list not filtered", s);
        return {};
      }
      while (*p == ',' || *p == ' ') p++;
    }
    // VGPU_DEVICE_GPU_IDS: the KFD gpu_ids of the same devices, in the same order.
    if (const char* g = getenv("VGPU_DEVICE_GPU_IDS")) {
      size_t i = 0;
      for (const char* q = g; *q && i < out.size();) {
        char* end = nullptr;
        unsigned long long v = strtoull(q, &end, 10);
        if (end == q) break;
        out[i++].gpu_id = v;
        q = end;
        while (*q == ',' || *q == ' ') q++;
      }
    }
    return out;
  }
  if (!attached) return out;
  const Region* r = shim().region.raw();
  for (int i = 0; i < kMaxDevices; i++)
    if (r->dev[i].configured)
      out.push_back({r->dev[i].domain, r->dev[i].bdf, r->dev[i].gpu_id ? r->dev[i].gpu_id : kNoGpuId});
  return out;
}

bool amdsmi_visible(amdsmi_processor_handle h, const std::vector<Bdf>& vis);

// Split duplicate vGPUs (VGPU_DUPLICATE_SPLIT): a GPU the device list names k times is listed
// k times - one entry per vGPU, as the container's HIP devices are (vdev_hooks.cpp).
int visible_times(amdsmi_processor_handle h, const std::vector<Bdf>& vis) {
  if (!amdsmi_visible(h, vis)) return 0;
  if (!config().duplicate_split) return 1;
  VGPU_REAL_IMPL(amdsmi_get_gpu_device_bdf, "libamd_smi", nullptr);
  amdsmi_bdf_t b;
  b.as_uint = 0;
  if (!real_amdsmi_get_gpu_device_bdf || real_amdsmi_get_gpu_device_bdf(h, &b) != AMDSMI_STATUS_SUCCESS) return 1;
  int k = 0;
  for (const Bdf& v : vis)
    if (v.domain == (b.as_uint >> 16) && v.bdfid == (uint32_t)(b.as_uint & 0xffff)) k++;
  return k > 0 ? k : 1;
}

bool amdsmi_visible(amdsmi_processor_handle h, const std::vector<Bdf>& vis) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_device_bdf, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_device_bdf) return true;
  amdsmi_bdf_t b;
  b.as_uint = 0;
  if (real_amdsmi_get_gpu_device_bdf(h, &b) != AMDSMI_STATUS_SUCCESS) return true;  // not a GPU: keep
  uint64_t gid = kNoGpuId;
  bool asked = false;
  for (const Bdf& v : vis) {
    if (v.domain != (b.as_uint >> 16) || v.bdfid != (uint32_t)(b.as_uint & 0xffff)) continue;
    if (v.gpu_id == kNoGpuId) return true;
    if (!asked) {
      gid = amdsmi_gpu_id(h);
      asked = true;
    }
    if (gid == kNoGpuId || gid == v.gpu_id) return true;  // partition of this container's GPU
  }
  return false;
}

int rsmi_dev(uint32_t idx) {
  VGPU_REAL_IMPL(rsmi_dev_pci_id_get, "librocm_smi64", nullptr);
  if (!real_rsmi_dev_pci_id_get) return -1;
  uint64_t id = 0;
  if (real_rsmi_dev_pci_id_get(idx, &id) != RSMI_STATUS_SUCCESS) return -1;
  // rocm_smi's "GUID" is the KFD gpu_id: it separates partitions at one PCI address.
  VGPU_REAL_IMPL(rsmi_dev_guid_get, "librocm_smi64", nullptr);
  uint64_t guid = kNoGpuId;
  if (!real_rsmi_dev_guid_get || real_rsmi_dev_guid_get(idx, &guid) != RSMI_STATUS_SUCCESS) guid = kNoGpuId;
  return device_by_bdf(id >> 32, (uint32_t)(id & 0xffff), guid);
}

void* rsmi_real(const char* name) { return resolve_real("librocm_smi64", name, nullptr); }

// The container's rocm_smi device indices: the node's indices of its GPUs, in the node's
// order. Identity when nothing is to be hidden (no visible-BDF list, VGPU_HOOK_SMI=0).
struct RsmiMap {
  std::mutex mu;
  bool built = false;
  bool identity = true;
  std::vector<uint32_t> phys;
};

RsmiMap& rsmi_map() {
  static RsmiMap* m = new RsmiMap();  // never destroyed: SMI calls may run during exit
  std::lock_guard<std::mutex> g(m->mu);
  if (m->built) return *m;
  std::vector<Bdf> vis = visible_bdfs();
  if (vis.empty()) return *m;  // nothing to hide (yet: a later GPU process may record its BDF)
  VGPU_REAL_IMPL(rsmi_num_monitor_devices, "librocm_smi64", nullptr);
  VGPU_REAL_IMPL(rsmi_dev_pci_id_get, "librocm_smi64", nullptr);
  uint32_t n = 0;
  if (!real_rsmi_num_monitor_devices || !real_rsmi_dev_pci_id_get ||
      real_rsmi_num_monitor_devices(&n) != RSMI_STATUS_SUCCESS)
    return *m;  // rsmi_init not called yet: identity for now, try again next call
  m->phys.clear();
  for (uint32_t i = 0; i < n; i++) {
    uint64_t id = 0;
    if (real_rsmi_dev_pci_id_get(i, &id) != RSMI_STATUS_SUCCESS) continue;
    // (split duplicate vGPUs: one index per entry of the device list naming this GPU)
    for (const Bdf& v : vis)
      if (v.domain == (id >> 32) && v.bdfid == (uint32_t)(id & 0xffff)) {
        m->phys.push_back(i);
        if (!config().duplicate_split) break;
      }
  }
  m->identity = false;
  m->built = true;
  return *m;
}

// Container index -> node index; false for an index the container does not have.
bool rsmi_phys(uint32_t v, uint32_t* p) {
  RsmiMap& m = rsmi_map();
  if (m.identity) {
    *p = v;
    return true;
  }
  if (v >= m.phys.size()) return false;
  *p = m.phys[v];
  return true;
}

struct RsmiRemap {
  const char* name;
  void* fn;
};

#include "rsmi_remap_gen.inc"

// Whether `pid` (a host PID, as the SMI libraries report them) is one of this
// container's GPU processes. Only a known host PID is compared; a slot's own PID stands
// in for it only when that PID lives in the host's namespace (no PID namespace: the two
// are the same number). Comparing a namespaced PID with host PIDs would let an unrelated
// process of another tenant that happens to have that number through the filter.
bool region_has_pid(uint32_t pid) {
  const Region* r = shim().region.raw();
  for (int i = 0; i < kMaxProcs; i++) {
    int32_t p = r->procs[i].pid.load(std::memory_order_relaxed);
    if (!p) continue;
    int32_t hp = r->procs[i].hostpid.load(std::memory_order_relaxed);
    if (hp > 0 ? (uint32_t)hp == pid : (r->procs[i].pidns == kInitPidNs && (uint32_t)p == pid)) return true;
  }
  return false;
}

}  // namespace

extern "C" {

amdsmi_status_t amdsmi_get_gpu_memory_total(amdsmi_processor_handle h, amdsmi_memory_type_t type, uint64_t* total) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_memory_total, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_memory_total) return AMDSMI_STATUS_NOT_SUPPORTED;
  amdsmi_status_t st = real_amdsmi_get_gpu_memory_total(h, type, total);
  if (st != AMDSMI_STATUS_SUCCESS || type != AMDSMI_MEM_TYPE_VRAM || !total) return st;
  int dev = amdsmi_dev(h);
  if (dev >= 0) *total = virt_total(dev, *total);
  return st;
}

amdsmi_status_t amdsmi_get_gpu_memory_usage(amdsmi_processor_handle h, amdsmi_memory_type_t type, uint64_t* used) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_memory_usage, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_memory_usage) return AMDSMI_STATUS_NOT_SUPPORTED;
  amdsmi_status_t st = real_amdsmi_get_gpu_memory_usage(h, type, used);
  if (st != AMDSMI_STATUS_SUCCESS || type != AMDSMI_MEM_TYPE_VRAM || !used) return st;
  int dev = amdsmi_dev(h);
  if (dev >= 0 && shim().region.limit(dev)) *used = virt_used(dev);
  return st;
}

amdsmi_status_t amdsmi_get_gpu_vram_usage(amdsmi_processor_handle h, amdsmi_vram_usage_t* info) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_vram_usage, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_vram_usage) return AMDSMI_STATUS_NOT_SUPPORTED;
  amdsmi_status_t st = real_amdsmi_get_gpu_vram_usage(h, info);
  if (st != AMDSMI_STATUS_SUCCESS || !info) return st;
  int dev = amdsmi_dev(h);
  if (dev >= 0 && shim().region.limit(dev)) {
    info->vram_total = (uint32_t)(virt_total(dev, (uint64_t)info->vram_total << 20) >> 20);
    info->vram_used = (uint32_t)(virt_used(dev) >> 20);
  }
  return st;
}

rsmi_status_t rsmi_dev_memory_total_get(uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* total) {
  VGPU_REAL_IMPL(rsmi_dev_memory_total_get, "librocm_smi64", nullptr);
  if (!real_rsmi_dev_memory_total_get) return RSMI_STATUS_NOT_SUPPORTED;
  if (!rsmi_phys(dv_ind, &dv_ind)) return RSMI_STATUS_INVALID_ARGS;
  rsmi_status_t st = real_rsmi_dev_memory_total_get(dv_ind, type, total);
  if (st != RSMI_STATUS_SUCCESS || type != RSMI_MEM_TYPE_VRAM || !total) return st;
  int dev = rsmi_dev(dv_ind);
  if (dev >= 0) *total = virt_total(dev, *total);
  return st;
}

rsmi_status_t rsmi_dev_memory_usage_get(uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* used) {
  VGPU_REAL_IMPL(rsmi_dev_memory_usage_get, "librocm_smi64", nullptr);
  if (!real_rsmi_dev_memory_usage_get) return RSMI_STATUS_NOT_SUPPORTED;
  if (!rsmi_phys(dv_ind, &dv_ind)) return RSMI_STATUS_INVALID_ARGS;
  rsmi_status_t st = real_rsmi_dev_memory_usage_get(dv_ind, type, used);
  if (st != RSMI_STATUS_SUCCESS || type != RSMI_MEM_TYPE_VRAM || !used) return st;
  int dev = rsmi_dev(dv_ind);
  if (dev >= 0 && shim().region.limit(dev)) *used = virt_used(dev);
  return st;
}

amdsmi_status_t amdsmi_get_processor_handles(amdsmi_socket_handle socket, uint32_t* count,
                                             amdsmi_processor_handle* handles) {
  VGPU_REAL_IMPL(amdsmi_get_processor_handles, "libamd_smi", nullptr);
  if (!real_amdsmi_get_processor_handles) return AMDSMI_STATUS_NOT_SUPPORTED;
  std::vector<Bdf> vis = visible_bdfs();
  if (vis.empty() || !count) return real_amdsmi_get_processor_handles(socket, count, handles);
  uint32_t n = 0;
  amdsmi_status_t st = real_amdsmi_get_processor_handles(socket, &n, nullptr);
  if (st != AMDSMI_STATUS_SUCCESS) return st;
  std::vector<amdsmi_processor_handle> all(n);
  if (n && (st = real_amdsmi_get_processor_handles(socket, &n, all.data())) != AMDSMI_STATUS_SUCCESS) return st;
  std::vector<amdsmi_processor_handle> mine;
  for (uint32_t i = 0; i < n && i < all.size(); i++)
    for (int k = visible_times(all[i], vis); k > 0; k--) mine.push_back(all[i]);
  if (!handles) {
    *count = (uint32_t)mine.size();
    return AMDSMI_STATUS_SUCCESS;
  }
  uint32_t cap = *count, w = 0;
  for (; w < cap && w < mine.size(); w++) handles[w] = mine[w];
  *count = cap < mine.size() ? (uint32_t)mine.size() : w;
  return AMDSMI_STATUS_SUCCESS;
}

amdsmi_status_t amdsmi_get_gpu_process_list(amdsmi_processor_handle h, uint32_t* max_processes,
                                            amdsmi_proc_info_t* list) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_process_list, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_process_list) return AMDSMI_STATUS_NOT_SUPPORTED;
  if (!config().hook_smi || !max_processes || !shim_attach_region_only())
    return real_amdsmi_get_gpu_process_list(h, max_processes, list);
  // The full list (host PIDs), then only this container's processes.
  std::vector<amdsmi_proc_info_t> all(64);
  amdsmi_status_t st;
  for (;;) {
    uint32_t n = (uint32_t)all.size();
    st = real_amdsmi_get_gpu_process_list(h, &n, all.data());
    if (st == AMDSMI_STATUS_OUT_OF_RESOURCES && n > all.size() && n < 65536) {
      all.resize(n);
      continue;
    }
    if (st != AMDSMI_STATUS_SUCCESS) return st;
    all.resize(n);
    break;
  }
  std::vector<amdsmi_proc_info_t> mine;
  for (const amdsmi_proc_info_t& p : all)
    if (region_has_pid(p.pid)) mine.push_back(p);
  const uint32_t cap = *max_processes;
  *max_processes = (uint32_t)mine.size();
  if (cap == 0 || !list) return AMDSMI_STATUS_SUCCESS;
  for (uint32_t i = 0; i < cap && i < mine.size(); i++) list[i] = mine[i];
  return cap < mine.size() ? AMDSMI_STATUS_OUT_OF_RESOURCES : AMDSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_compute_process_info_get(rsmi_process_info_t* procs, uint32_t* num_items) {
  VGPU_REAL_IMPL(rsmi_compute_process_info_get, "librocm_smi64", nullptr);
  if (!real_rsmi_compute_process_info_get) return RSMI_STATUS_NOT_SUPPORTED;
  if (!config().hook_smi || !num_items || !shim_attach_region_only())
    return real_rsmi_compute_process_info_get(procs, num_items);
  std::vector<rsmi_process_info_t> all(64);
  for (;;) {
    uint32_t n = (uint32_t)all.size();
    rsmi_status_t st = real_rsmi_compute_process_info_get(all.data(), &n);
    if (st == RSMI_STATUS_INSUFFICIENT_SIZE && all.size() < 65536) {
      all.resize(all.size() * 4);
      continue;
    }
    if (st != RSMI_STATUS_SUCCESS) return st;
    all.resize(n);
    break;
  }
  std::vector<rsmi_process_info_t> mine;
  for (const rsmi_process_info_t& p : all)
    if (region_has_pid(p.process_id)) mine.push_back(p);
  // rocm_smi's contract: a null array asks for the count; otherwise fill up to
  // *num_items, report how many were written, INSUFFICIENT_SIZE if some did not fit.
  if (!procs) {
    *num_items = (uint32_t)mine.size();
    return RSMI_STATUS_SUCCESS;
  }
  const uint32_t cap = *num_items;
  uint32_t w = 0;
  for (; w < cap && w < mine.size(); w++) procs[w] = mine[w];
  *num_items = w;
  return w < mine.size() ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_num_monitor_devices(uint32_t* num_devices) {
  VGPU_REAL_IMPL(rsmi_num_monitor_devices, "librocm_smi64", nullptr);
  if (!real_rsmi_num_monitor_devices) return RSMI_STATUS_NOT_SUPPORTED;
  rsmi_status_t st = real_rsmi_num_monitor_devices(num_devices);
  if (st != RSMI_STATUS_SUCCESS || !num_devices) return st;
  RsmiMap& m = rsmi_map();
  if (!m.identity) *num_devices = (uint32_t)m.phys.size();
  return st;
}

// The GPUs a process uses, as container indices (GPUs outside the container dropped).
rsmi_status_t rsmi_compute_process_gpus_get(uint32_t pid, uint32_t* dv_indices, uint32_t* num_devices) {
  VGPU_REAL_IMPL(rsmi_compute_process_gpus_get, "librocm_smi64", nullptr);
  if (!real_rsmi_compute_process_gpus_get) return RSMI_STATUS_NOT_SUPPORTED;
  RsmiMap& m = rsmi_map();
  if (m.identity || !num_devices) return real_rsmi_compute_process_gpus_get(pid, dv_indices, num_devices);
  std::vector<uint32_t> all(64);
  rsmi_status_t st;
  for (;;) {
    uint32_t n = (uint32_t)all.size();
    st = real_rsmi_compute_process_gpus_get(pid, all.data(), &n);
    if (st == RSMI_STATUS_INSUFFICIENT_SIZE && all.size() < 4096) {
      all.resize(all.size() * 4);
      continue;
    }
    if (st != RSMI_STATUS_SUCCESS) return st;
    all.resize(std::min<size_t>(n, all.size()));
    break;
  }
  std::vector<uint32_t> mine;
  for (uint32_t p : all)
    for (size_t v = 0; v < m.phys.size(); v++)
      if (m.phys[v] == p) mine.push_back((uint32_t)v);
  const uint32_t cap = *num_devices;
  *num_devices = (uint32_t)mine.size();
  if (!dv_indices) return RSMI_STATUS_SUCCESS;
  for (uint32_t i = 0; i < cap && i < mine.size(); i++) dv_indices[i] = mine[i];
  return cap < mine.size() ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_compute_process_info_by_pid_get(uint32_t pid, rsmi_process_info_t* proc) {
  VGPU_REAL_IMPL(rsmi_compute_process_info_by_pid_get, "librocm_smi64", nullptr);
  if (!real_rsmi_compute_process_info_by_pid_get) return RSMI_STATUS_NOT_SUPPORTED;
  if (config().hook_smi && shim_attach_region_only() && !region_has_pid(pid)) return RSMI_STATUS_NOT_FOUND;
  return real_rsmi_compute_process_info_by_pid_get(pid, proc);
}

}  // extern "C"

namespace vgpu {
// dlsym_hook.cpp: the index-remapping wrapper for a rocm_smi entry point, or null.
void* rsmi_remap_hook(const char* name) {
  for (const RsmiRemap& r : kRsmiRemap)
    if (strcmp(r.name, name) == 0) return r.fn;
  return nullptr;
}
}  // namespace vgpu
