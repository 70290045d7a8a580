// A fake librocm_smi64.so for CPU-only tests of the shim's rocm_smi virtualisation
// (tests/test_rsmi_remap.py): four GPUs whose answers encode their node index, so a test
// can see which physical device a container-index call reached.
//   GPU i: PCI 0000:(0x05 + 0x10 i):00.0, device id 0x1000 + i, (i + 1) GiB of VRAM,
//   link weight src -> dst = 10 src + dst; every process uses all four GPUs.
#include <rocm_smi/rocm_smi.h>

#include <cstdio>

namespace {
constexpr uint32_t kGpus = 4;
}

extern "C" {

rsmi_status_t rsmi_init(uint64_t) { return RSMI_STATUS_SUCCESS; }
rsmi_status_t rsmi_shut_down() { return RSMI_STATUS_SUCCESS; }

rsmi_status_t rsmi_num_monitor_devices(uint32_t* n) {
  if (!n) return RSMI_STATUS_INVALID_ARGS;
  *n = kGpus;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_pci_id_get(uint32_t i, uint64_t* id) {
  if (i >= kGpus || !id) return RSMI_STATUS_INVALID_ARGS;
  *id = (uint64_t)(0x05 + 0x10 * i) << 8;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_id_get(uint32_t i, uint16_t* id) {
  if (i >= kGpus || !id) return RSMI_STATUS_INVALID_ARGS;
  *id = (uint16_t)(0x1000 + i);
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_name_get(uint32_t i, char* name, size_t len) {
  if (i >= kGpus || !name) return RSMI_STATUS_INVALID_ARGS;
  snprintf(name, len, "fake-gpu-%u", i);
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_dev_memory_total_get(uint32_t i, rsmi_memory_type_t, uint64_t* total) {
  if (i >= kGpus || !total) return RSMI_STATUS_INVALID_ARGS;
  *total = (uint64_t)(i + 1) << 30;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_topo_get_link_weight(uint32_t src, uint32_t dst, uint64_t* weight) {
  if (src >= kGpus || dst >= kGpus || !weight) return RSMI_STATUS_INVALID_ARGS;
  *weight = 10ull * src + dst;
  return RSMI_STATUS_SUCCESS;
}

rsmi_status_t rsmi_compute_process_gpus_get(uint32_t, uint32_t* idx, uint32_t* n) {
  if (!n) return RSMI_STATUS_INVALID_ARGS;
  const uint32_t cap = *n;
  *n = kGpus;
  if (!idx) return RSMI_STATUS_SUCCESS;
  for (uint32_t i = 0; i < cap && i < kGpus; i++) idx[i] = i;
  return cap < kGpus ? RSMI_STATUS_INSUFFICIENT_SIZE : RSMI_STATUS_SUCCESS;
}

}  // extern "C"
