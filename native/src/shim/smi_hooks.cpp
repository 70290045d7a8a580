// amd-smi / rocm-smi memory virtualisation (in-container tools show the vGPU quota).
//
// Reference: src/nvml/hook.c nvmlDeviceGetMemoryInfo(_v2) [327-361] reports
// total = limit, used = region usage (or the monitor value under MEMORY_OVERRIDE),
// free = limit - used. The MI355X equivalents are amdsmi_get_gpu_memory_total/usage,
// amdsmi_get_gpu_vram_usage and the rocm_smi rsmi_dev_memory_total/usage_get calls.
// These run in processes that usually never initialise ROCr (amd-smi itself), so
// the region is attached read-mostly and devices are matched by PCI BDF, which the
// first GPU process of the container recorded in the region.
#include <amd_smi/amdsmi.h>
#include <rocm_smi/rocm_smi.h>

#include "real.h"
#include "shim.h"
#include "vgpu/log.h"

using namespace vgpu;

namespace {

// Region device index for a PCI (domain, bdfid) pair, or -1.
int device_by_bdf(uint64_t domain, uint32_t bdfid) {
  if (!shim_attach_region_only()) return -1;
  if (!config().hook_smi) return -1;
  const Region* r = shim().region.raw();
  for (int i = 0; i < kMaxDevices; i++) {
    const DeviceState& d = r->dev[i];
    if (d.configured && d.bdf == bdfid && d.domain == (uint32_t)domain) return i;
  }
  return -1;
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

int amdsmi_dev(amdsmi_processor_handle h) {
  VGPU_REAL_IMPL(amdsmi_get_gpu_device_bdf, "libamd_smi", nullptr);
  if (!real_amdsmi_get_gpu_device_bdf) return -1;
  amdsmi_bdf_t b;
  b.as_uint = 0;
  if (real_amdsmi_get_gpu_device_bdf(h, &b) != AMDSMI_STATUS_SUCCESS) return -1;
  return device_by_bdf(b.as_uint >> 16, (uint32_t)(b.as_uint & 0xffff));
}

int rsmi_dev(uint32_t idx) {
  VGPU_REAL_IMPL(rsmi_dev_pci_id_get, "librocm_smi64", nullptr);
  if (!real_rsmi_dev_pci_id_get) return -1;
  uint64_t id = 0;
  if (real_rsmi_dev_pci_id_get(idx, &id) != RSMI_STATUS_SUCCESS) return -1;
  return device_by_bdf(id >> 32, (uint32_t)(id & 0xffff));
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
  rsmi_status_t st = real_rsmi_dev_memory_total_get(dv_ind, type, total);
  if (st != RSMI_STATUS_SUCCESS || type != RSMI_MEM_TYPE_VRAM || !total) return st;
  int dev = rsmi_dev(dv_ind);
  if (dev >= 0) *total = virt_total(dev, *total);
  return st;
}

rsmi_status_t rsmi_dev_memory_usage_get(uint32_t dv_ind, rsmi_memory_type_t type, uint64_t* used) {
  VGPU_REAL_IMPL(rsmi_dev_memory_usage_get, "librocm_smi64", nullptr);
  if (!real_rsmi_dev_memory_usage_get) return RSMI_STATUS_NOT_SUPPORTED;
  rsmi_status_t st = real_rsmi_dev_memory_usage_get(dv_ind, type, used);
  if (st != RSMI_STATUS_SUCCESS || type != RSMI_MEM_TYPE_VRAM || !used) return st;
  int dev = rsmi_dev(dv_ind);
  if (dev >= 0 && shim().region.limit(dev)) *used = virt_used(dev);
  return st;
}

}  // extern "C"
