// Split duplicate vGPUs: two vGPUs of one physical GPU as two HIP devices of the container.
//
// Reference: its shim keeps a container's duplicate vGPUs apart as separate virtual devices
// with virtual PCI bus ids (`assigning_virtual_pcibusID` [device.c:81-117], the device map
// [nvml/util.c:135-162], NVIDIA_DEVICE_MAP server.go:490,493) and disables cooperative launch
// on them [device.c:130-134]. ROCm enumerates one device per GPU agent, so with the plugin's
// default --duplicate-vgpus=split (VGPU_DUPLICATE_SPLIT=1) the shim presents them as separate
// devices at the HIP layer (=merge: one device, summed quota and CU share; docs/ABI.md
// "Duplicate vGPUs"):
//
//   * hipGetDeviceCount counts every vGPU; virtual device v is backed by physical device
//     phys(v) (the vGPUs of one GPU are consecutive, in VGPU_DEVICE_MAP order);
//   * hipSetDevice(v) selects phys(v) and remembers v for the thread (hipGetDevice returns
//     it), so torch.cuda.set_device(1), a cuda:1 tensor or one rank per visible device work;
//   * every entry point that takes a device ordinal maps it (hip_gates.def `device` rows for
//     the generic ones, the hooks below for those that return or virtualise something);
//   * each virtual device has its own quota: a region slot after the agents' (which keep the
//     summed quota as the physical guard), charged by the HSA allocation hook for the calling
//     thread's virtual device (hsa_hooks.cpp), reported by hipMemGetInfo / hipDeviceTotalMem /
//     the device properties;
//   * peer access between two virtual devices of one GPU is the same memory: reported
//     possible and enabled without a runtime call; cooperative launch stays as the runtime
//     reports it (one GPU).
// CU masks and the GPU-time limiter stay per physical GPU (HIP's hardware queues are shared by
// all streams of a device), with the vGPUs' shares summed as in merge mode. RCCL between the
// virtual devices of one GPU is not supported (it sees one PCI address twice).
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <hip/hip_deprecated.h>  // hipDeviceProp_tR0000: the hip_4.2 hipGetDeviceProperties

#include <atomic>
#include <cstdint>
#include <cstring>
#include <mutex>

#include "real.h"
#include "shim.h"
#include "vgpu/devmap.h"
#include "vgpu/log.h"

using namespace vgpu;

namespace {

struct VirtDev {
  int phys = 0;    // HIP ordinal of the backing device
  int agent = 0;   // its agent (region device) index
  int slot = -1;   // region slot with this vGPU's quota (-1: the agent's own, no split)
};

std::atomic<int> g_state{0};  // 0 = not built, 1 = split active, 2 = off
VirtDev g_virt[kMaxDevices];
int g_nvirt = 0;
std::mutex g_build_mu;
thread_local int t_vdev = -1;  // the thread's current virtual device (-1 = none selected)

int real_device_count() {
  VGPU_REAL_HIP(hipGetDeviceCount);
  int n = 0;
  if (!real_hipGetDeviceCount || real_hipGetDeviceCount(&n) != hipSuccess) return -1;
  return n;
}

// Builds the virtual device table once the shim is initialised (the region holds the
// virtual slots' quotas). Off when the config asks for no split or has no duplicates.
bool build() {
  int st = g_state.load(std::memory_order_acquire);
  if (__builtin_expect(st != 0, 1)) return st == 1;
  // The shim's configuration is read when it initialises (with ROCr): a program whose first
  // HIP call takes a device ordinal (hipSetDevice(1), hipGetDeviceProperties) gets here first.
  ShimState& s = shim();
  if (s.phase.load(std::memory_order_acquire) == 0) (void)real_device_count();  // HIP (and the shim) initialise
  const int ph = s.phase.load(std::memory_order_acquire);
  if (ph == 3) {
    g_state.store(2, std::memory_order_release);  // inert shim: no limits, nothing to split
    return false;
  }
  if (ph != 2 || !s.active) return false;  // not yet: asked again on the next call
  const Config& cfg = config();
  if (!cfg.duplicate_split) {
    g_state.store(2, std::memory_order_release);
    return false;
  }
  std::lock_guard<std::mutex> g(g_build_mu);
  if ((st = g_state.load()) != 0) return st == 1;
  DeviceMap map;
  if (!parse_device_map(cfg.device_map.c_str(), &map) || map.duplicates == 0) {
    g_state.store(2, std::memory_order_release);
    return false;
  }
  const int np = real_device_count();
  if (np <= 0) return false;
  // Region slots of the virtual devices: after the agents, agent by agent, in map order
  // (shim.cpp assigns the same slots when it sets up the region).
  int first_slot[kMaxDevices], count[kMaxDevices] = {};
  for (int a = 0, next = s.n_agents; a < s.n_agents; a++) {
    char au[64];
    normalize_uuid(s.agents[a].uuid, au, sizeof(au));
    first_slot[a] = next;
    for (int j = 0; j < map.n; j++) {
      char mu[64];
      normalize_uuid(map.e[j].uuid, mu, sizeof(mu));
      if (!strcmp(mu, au)) count[a]++;
    }
    if (count[a] > 1) next += count[a];
  }
  int n = 0;
  for (int h = 0; h < np && n < kMaxDevices; h++) {
    const int a = hip_device_agent(h);
    const int c = count[a] > 1 ? count[a] : 1;
    for (int k = 0; k < c && n < kMaxDevices; k++) g_virt[n++] = VirtDev{h, a, count[a] > 1 ? first_slot[a] + k : -1};
  }
  g_nvirt = n;
  VLOG_INFO("duplicate vGPUs split: %d HIP device(s) over %d physical", n, np);
  g_state.store(1, std::memory_order_release);
  return true;
}

inline bool split() {
  const int st = g_state.load(std::memory_order_relaxed);
  return st == 1 || (st == 0 && build());
}

// The virtual device a physical ordinal stands for in the calling thread: its current one
// when that is backed by `phys`, else the first one backed by it.
int virt_of(int phys) {
  if (t_vdev >= 0 && t_vdev < g_nvirt && g_virt[t_vdev].phys == phys) return t_vdev;
  for (int v = 0; v < g_nvirt; v++)
    if (g_virt[v].phys == phys) return v;
  return phys;
}

int current_virt() {
  VGPU_REAL_HIP(hipGetDevice);
  int p = 0;
  if (real_hipGetDevice) (void)real_hipGetDevice(&p);
  return virt_of(p);
}

// The quota of virtual device v: its slot's limit and usage (0 limit = none).
void slot_quota(int v, uint64_t* limit, uint64_t* used) {
  ShimState& s = shim();
  const int slot = g_virt[v].slot;
  if (slot < 0) {
    *limit = *used = 0;
    return;
  }
  *limit = s.region.limit(slot);
  *used = s.region.usage(slot);
}

}  // namespace

namespace vgpu {

bool vdev_split_active() { return split(); }

int vdev_to_phys(int v) {
  if (v < 0 || !split() || v >= g_nvirt) return v;
  return g_virt[v].phys;
}

int vdev_charge_slot(int dev) {
  // Called from the HSA allocation hook, possibly inside the runtime's own initialisation:
  // only the table built already, and the thread's own record (no HIP call).
  if (g_state.load(std::memory_order_acquire) != 1) return -1;
  const int v = t_vdev;
  if (v >= 0 && v < g_nvirt && g_virt[v].agent == dev) return g_virt[v].slot;
  for (int i = 0; i < g_nvirt; i++)
    if (g_virt[i].agent == dev) return g_virt[i].slot;
  return -1;
}

}  // namespace vgpu

extern "C" {

hipError_t hipGetDeviceCount(int* count) {
  VGPU_REAL_HIP(hipGetDeviceCount);
  if (!real_hipGetDeviceCount) return hipErrorNotSupported;
  hipError_t e = real_hipGetDeviceCount(count);
  if (e == hipSuccess && count && split()) *count = g_nvirt;
  return e;
}

hipError_t hipSetDevice(int device) {
  VGPU_REAL_HIP(hipSetDevice);
  if (!real_hipSetDevice) return hipErrorNotSupported;
  if (!split()) return real_hipSetDevice(device);
  if (device < 0 || device >= g_nvirt) return hipErrorInvalidDevice;
  hipError_t e = real_hipSetDevice(g_virt[device].phys);
  if (e == hipSuccess) t_vdev = device;
  return e;
}

hipError_t hipGetDevice(int* device) {
  VGPU_REAL_HIP(hipGetDevice);
  if (!real_hipGetDevice) return hipErrorNotSupported;
  hipError_t e = real_hipGetDevice(device);
  if (e == hipSuccess && device && split()) *device = virt_of(*device);
  return e;
}

hipError_t hipDeviceGet(hipDevice_t* device, int ordinal) {
  VGPU_REAL_HIP(hipDeviceGet);
  if (!real_hipDeviceGet) return hipErrorNotSupported;
  if (!split()) return real_hipDeviceGet(device, ordinal);
  if (ordinal < 0 || ordinal >= g_nvirt) return hipErrorInvalidDevice;
  hipError_t e = real_hipDeviceGet(device, g_virt[ordinal].phys);
  if (e == hipSuccess && device) *device = ordinal;  // HIP's device handle is the ordinal
  return e;
}

hipError_t hipStreamGetDevice(hipStream_t stream, hipDevice_t* device) {
  VGPU_REAL_HIP(hipStreamGetDevice);
  if (!real_hipStreamGetDevice) return hipErrorNotSupported;
  hipError_t e = real_hipStreamGetDevice(stream, device);
  if (e == hipSuccess && device && split()) *device = virt_of(*device);
  return e;
}

hipError_t hipDeviceGetByPCIBusId(int* device, const char* pci_bus_id) {
  VGPU_REAL_HIP(hipDeviceGetByPCIBusId);
  if (!real_hipDeviceGetByPCIBusId) return hipErrorNotSupported;
  hipError_t e = real_hipDeviceGetByPCIBusId(device, pci_bus_id);
  if (e == hipSuccess && device && split()) *device = virt_of(*device);
  return e;
}

#undef hipGetDeviceProperties
hipError_t hipGetDeviceProperties(hipDeviceProp_tR0000* prop, int device) {
  using Fn = hipError_t (*)(hipDeviceProp_tR0000*, int);
  VGPU_REAL_AS(hipGetDeviceProperties, Fn, "libamdhip64", "hip_4.2");
  if (!real_hipGetDeviceProperties) return hipErrorNotSupported;
  if (!split()) return real_hipGetDeviceProperties(prop, device);
  if (device < 0 || device >= g_nvirt) return hipErrorInvalidDevice;
  hipError_t e = real_hipGetDeviceProperties(prop, g_virt[device].phys);
  uint64_t lim = 0, used = 0;
  slot_quota(device, &lim, &used);
  if (e == hipSuccess && prop && lim) prop->totalGlobalMem = lim;
  return e;
}

hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int device) {
  VGPU_REAL_HIP(hipGetDevicePropertiesR0600);
  if (!real_hipGetDevicePropertiesR0600) return hipErrorNotSupported;
  if (!split()) return real_hipGetDevicePropertiesR0600(prop, device);
  if (device < 0 || device >= g_nvirt) return hipErrorInvalidDevice;
  hipError_t e = real_hipGetDevicePropertiesR0600(prop, g_virt[device].phys);
  uint64_t lim = 0, used = 0;
  slot_quota(device, &lim, &used);
  if (e == hipSuccess && prop && lim) prop->totalGlobalMem = lim;
  return e;
}

// Device attributes of virtual device v: the backing GPU's, except its global memory, which is
// v's own quota (hipDeviceAttributeTotalGlobalMem is an int: a quota past INT32_MAX saturates,
// as the runtime saturates the whole 288 GB GPU: profiles/r6y).
hipError_t hipDeviceGetAttribute(int* value, hipDeviceAttribute_t attr, int device) {
  VGPU_REAL_HIP(hipDeviceGetAttribute);
  if (!real_hipDeviceGetAttribute) return hipErrorNotSupported;
  if (!split()) return real_hipDeviceGetAttribute(value, attr, device);
  if (device < 0 || device >= g_nvirt) return hipErrorInvalidDevice;
  hipError_t e = real_hipDeviceGetAttribute(value, attr, g_virt[device].phys);
  if (e != hipSuccess || !value || attr != hipDeviceAttributeTotalGlobalMem) return e;
  uint64_t lim = 0, used = 0;
  slot_quota(device, &lim, &used);
  if (lim) *value = lim > (uint64_t)INT32_MAX ? INT32_MAX : (int)lim;
  return e;
}

hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t device) {
  VGPU_REAL_HIP(hipDeviceTotalMem);
  if (!real_hipDeviceTotalMem) return hipErrorNotSupported;
  if (!split()) return real_hipDeviceTotalMem(bytes, device);
  if (device < 0 || device >= g_nvirt) return hipErrorInvalidDevice;
  hipError_t e = real_hipDeviceTotalMem(bytes, g_virt[device].phys);
  uint64_t lim = 0, used = 0;
  slot_quota(device, &lim, &used);
  if (e == hipSuccess && bytes && lim) *bytes = lim;
  return e;
}

// The current device's free and total memory: the runtime's answer (the physical GPU, within
// the summed quota of its vGPUs: the HSA hook), narrowed to the current virtual device's own.
hipError_t hipMemGetInfo(size_t* free_bytes, size_t* total_bytes) {
  VGPU_REAL_HIP(hipMemGetInfo);
  if (!real_hipMemGetInfo) return hipErrorNotSupported;
  hipError_t e = real_hipMemGetInfo(free_bytes, total_bytes);
  if (e != hipSuccess || !split()) return e;
  const int v = current_virt();
  if (v < 0 || v >= g_nvirt) return e;
  uint64_t lim = 0, used = 0;
  slot_quota(v, &lim, &used);
  if (!lim) return e;
  const uint64_t left = lim > used ? lim - used : 0;
  if (free_bytes && *free_bytes > left) *free_bytes = left;
  if (total_bytes) *total_bytes = lim;
  return e;
}

hipError_t hipDeviceCanAccessPeer(int* can, int device, int peer) {
  VGPU_REAL_HIP(hipDeviceCanAccessPeer);
  if (!real_hipDeviceCanAccessPeer) return hipErrorNotSupported;
  if (!split()) return real_hipDeviceCanAccessPeer(can, device, peer);
  if (device < 0 || device >= g_nvirt || peer < 0 || peer >= g_nvirt) return hipErrorInvalidDevice;
  if (g_virt[device].phys == g_virt[peer].phys) {
    if (can) *can = device != peer;  // one GPU's memory: always reachable (not from itself, as CUDA)
    return hipSuccess;
  }
  return real_hipDeviceCanAccessPeer(can, g_virt[device].phys, g_virt[peer].phys);
}

hipError_t hipDeviceEnablePeerAccess(int peer, unsigned int flags) {
  VGPU_REAL_HIP(hipDeviceEnablePeerAccess);
  if (!real_hipDeviceEnablePeerAccess) return hipErrorNotSupported;
  if (!split()) return real_hipDeviceEnablePeerAccess(peer, flags);
  if (peer < 0 || peer >= g_nvirt) return hipErrorInvalidDevice;
  const int cur = current_virt();
  if (cur >= 0 && cur < g_nvirt && g_virt[cur].phys == g_virt[peer].phys) return hipSuccess;  // same memory
  return real_hipDeviceEnablePeerAccess(g_virt[peer].phys, flags);
}

hipError_t hipDeviceDisablePeerAccess(int peer) {
  VGPU_REAL_HIP(hipDeviceDisablePeerAccess);
  if (!real_hipDeviceDisablePeerAccess) return hipErrorNotSupported;
  if (!split()) return real_hipDeviceDisablePeerAccess(peer);
  if (peer < 0 || peer >= g_nvirt) return hipErrorInvalidDevice;
  const int cur = current_virt();
  if (cur >= 0 && cur < g_nvirt && g_virt[cur].phys == g_virt[peer].phys) return hipSuccess;
  return real_hipDeviceDisablePeerAccess(g_virt[peer].phys);
}

}  // extern "C"
