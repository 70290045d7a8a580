// A fake libamdhip64.so over the fake ROCr (fake_hsa.cpp) for CPU-only shim tests.
//
// Implements the slice of the HIP API the shim interposes or calls: devices, hipMalloc /
// hipFree / hipMemGetInfo (through the HSA pool and agent-info entry points, as CLR does),
// streams (one HSA queue each, so the shim's CU masks land on them), and kernel launches
// executed by a per-device "GPU" thread that sleeps for the kernel's duration while
// reporting resident waves in the fake KFD cu_occupancy file. A kernel is a pointer to a
// uint32 duration in microseconds (the `function_address` argument of hipLaunchKernel;
// the graph-exec handle of hipGraphLaunch).
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>

#include <dlfcn.h>

#include <chrono>
#include <cstdlib>
#include <cstring>
#include <string>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <set>
#include <thread>

extern "C" int fake_rocr_set_occupancy(int dev, int cus);
extern "C" void fake_rocr_queue_submit(hsa_queue_t* queue);
extern "C" void fake_rocr_queue_retire(hsa_queue_t* queue);

namespace {

struct Device {
  hsa_agent_t agent{0};
  int rocr = 0;  // index among the fake ROCr's GPU agents (HIP_VISIBLE_DEVICES may reorder)
  hsa_amd_memory_pool_t pool{0};
  std::mutex mu;
  std::condition_variable cv;
  std::deque<std::pair<uint32_t, hsa_queue_t*>> work;  // kernel durations (µs) and their stream's queue
  bool running = false;
  uint64_t busy_us = 0;
  uint64_t kernels = 0;
  std::thread th;
};

std::mutex g_mu;
bool g_inited = false;
int g_n = 0;
// Never destroyed: the per-device GPU threads wait on these until the process ends.
Device* const g_dev = new Device[16];
thread_local int t_dev = 0;

void gpu_loop(int d) {
  Device& D = g_dev[d];
  for (;;) {
    uint32_t us;
    hsa_queue_t* q;
    {
      std::unique_lock<std::mutex> l(D.mu);
      D.cv.wait(l, [&] { return !D.work.empty(); });
      us = D.work.front().first;
      q = D.work.front().second;
      if (!D.running) fake_rocr_set_occupancy(D.rocr, 64);
      D.running = true;
    }
    auto t0 = std::chrono::steady_clock::now();
    std::this_thread::sleep_for(std::chrono::microseconds(us));
    uint64_t took = (uint64_t)std::chrono::duration_cast<std::chrono::microseconds>(
                        std::chrono::steady_clock::now() - t0).count();
    std::lock_guard<std::mutex> l(D.mu);
    if (q) fake_rocr_queue_retire(q);
    D.work.pop_front();
    D.busy_us += took;  // the time the "GPU" was really busy (sleeps overshoot)
    D.kernels++;
    if (D.work.empty()) {
      D.running = false;
      fake_rocr_set_occupancy(D.rocr, 0);
      D.cv.notify_all();
    }
  }
}

hsa_agent_t g_all[16];
int g_nall = 0;
hsa_agent_t g_cpu{0};
hsa_amd_memory_pool_t g_cpu_pool{0};  // pinned host memory comes from here, as in CLR

hsa_status_t agent_cb(hsa_agent_t a, void*) {
  hsa_device_type_t t;
  hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
  if (t == HSA_DEVICE_TYPE_GPU && g_nall < 16) g_all[g_nall++] = a;
  if (t == HSA_DEVICE_TYPE_CPU && !g_cpu.handle) g_cpu = a;
  return HSA_STATUS_SUCCESS;
}

// HIP devices over the ROCr agents, in HIP_VISIBLE_DEVICES order when it is set (as CLR).
void map_devices() {
  const char* v = getenv("HIP_VISIBLE_DEVICES");
  if (!v || !*v) {
    for (int i = 0; i < g_nall; i++) g_dev[g_n].rocr = i, g_dev[g_n++].agent = g_all[i];
    return;
  }
  for (const char* p = v; *p && g_n < 16;) {
    int i = atoi(p);
    if (i >= 0 && i < g_nall) g_dev[g_n].rocr = i, g_dev[g_n++].agent = g_all[i];
    while (*p && *p != ',') p++;
    if (*p == ',') p++;
  }
}

hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* data) {
  *static_cast<hsa_amd_memory_pool_t*>(data) = p;
  return HSA_STATUS_SUCCESS;
}

void init() {
  std::lock_guard<std::mutex> g(g_mu);
  if (g_inited) return;
  hsa_init();  // the shim's hsa_init hook runs here, as inside CLR
  hsa_iterate_agents(agent_cb, nullptr);
  map_devices();
  if (g_cpu.handle) hsa_amd_agent_iterate_memory_pools(g_cpu, pool_cb, &g_cpu_pool);
  for (int i = 0; i < g_n; i++) {
    hsa_amd_agent_iterate_memory_pools(g_dev[i].agent, pool_cb, &g_dev[i].pool);
    g_dev[i].th = std::thread(gpu_loop, i);
    g_dev[i].th.detach();
  }
  g_inited = true;
}

struct FakeStream {
  hsa_queue_t* q;
  int dev;
};

int dev_of(hipStream_t s) { return s ? reinterpret_cast<FakeStream*>(s)->dev : t_dev; }
hsa_queue_t* queue_of(hipStream_t s) { return s ? reinterpret_cast<FakeStream*>(s)->q : nullptr; }

void submit(int d, uint32_t us, hsa_queue_t* q) {
  Device& D = g_dev[d];
  std::lock_guard<std::mutex> l(D.mu);
  if (q) fake_rocr_queue_submit(q);
  D.work.push_back({us, q});
  D.cv.notify_all();
}

}  // namespace

extern "C" {

hipError_t hipInit(unsigned int) {
  init();
  return hipSuccess;
}

hipError_t hipGetDeviceCount(int* n) {
  init();
  *n = g_n;
  return hipSuccess;
}

hipError_t hipSetDevice(int d) {
  init();
  if (d < 0 || d >= g_n) return hipErrorInvalidDevice;
  t_dev = d;
  return hipSuccess;
}

hipError_t hipGetDevice(int* d) {
  init();
  *d = t_dev;
  return hipSuccess;
}

void fake_hip_record(const char* name);

hipError_t hipDeviceGetAttribute(int* value, hipDeviceAttribute_t attr, int d) {
  init();
  fake_hip_record("hipDeviceGetAttribute");
  if (!value || d < 0 || d >= g_n) return hipErrorInvalidDevice;
  uint32_t bdf = 0, dom = 0;
  hsa_agent_get_info(g_dev[d].agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_BDFID, &bdf);
  hsa_agent_get_info(g_dev[d].agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_DOMAIN, &dom);
  switch (attr) {
    case hipDeviceAttributePciBusId: *value = (int)(bdf >> 8); return hipSuccess;
    case hipDeviceAttributePciDeviceId: *value = (int)((bdf >> 3) & 0x1f); return hipSuccess;
    case hipDeviceAttributePciDomainId: *value = (int)dom; return hipSuccess;
    case hipDeviceAttributeTotalGlobalMem: {  // CLR: the pool size, saturated to an int
      size_t total = 0;
      hsa_amd_memory_pool_get_info(g_dev[d].pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &total);
      *value = total > (size_t)INT32_MAX ? INT32_MAX : (int)total;
      return hipSuccess;
    }
    default: return hipErrorInvalidValue;
  }
}

hipError_t hipMalloc(void** ptr, size_t size) {
  init();
  hsa_status_t s = hsa_amd_memory_pool_allocate(g_dev[t_dev].pool, size, 0, ptr);
  return s == HSA_STATUS_SUCCESS ? hipSuccess : hipErrorOutOfMemory;
}

hipError_t hipFree(void* ptr) {
  if (!ptr) return hipSuccess;
  // Device and pinned host memory alike are pool allocations (CLR frees both here).
  return hsa_amd_memory_pool_free(ptr) == HSA_STATUS_SUCCESS ? hipSuccess : hipErrorInvalidValue;
}

void fake_hip_record(const char* name);

// CLR exports a buffer through ROCr's IPC (hsa_amd_ipc_memory_create), which fails for memory
// that is no ROCr allocation.
hipError_t hipIpcGetMemHandle(hipIpcMemHandle_t* handle, void* ptr) {
  init();
  fake_hip_record("hipIpcGetMemHandle");
  if (!handle || !ptr) return hipErrorInvalidValue;
  hsa_amd_ipc_memory_t h;
  if (hsa_amd_ipc_memory_create(ptr, 0, &h) != HSA_STATUS_SUCCESS) return hipErrorInvalidDevicePointer;
  memset(handle, 0, sizeof(*handle));
  memcpy(handle, &h, sizeof(h) < sizeof(*handle) ? sizeof(h) : sizeof(*handle));
  return hipSuccess;
}

hipError_t hipMemGetInfo(size_t* free_b, size_t* total_b) {
  init();
  uint64_t avail = 0;
  size_t total = 0;
  hsa_agent_get_info(g_dev[t_dev].agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_MEMORY_AVAIL, &avail);
  hsa_amd_memory_pool_get_info(g_dev[t_dev].pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &total);
  *free_b = avail;
  *total_b = total;
  return hipSuccess;
}

hipError_t hipGetDevicePropertiesR0600(hipDeviceProp_tR0600* prop, int d) {
  init();
  if (!prop || d < 0 || d >= g_n) return hipErrorInvalidDevice;
  memset(prop, 0, sizeof(*prop));
  snprintf(prop->name, sizeof(prop->name), "fake gfx950 %d", d);
  size_t total = 0;
  hsa_amd_memory_pool_get_info(g_dev[d].pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, &total);
  prop->totalGlobalMem = total;
  prop->multiProcessorCount = 256;
  return hipSuccess;
}

hipError_t hipDeviceTotalMem(size_t* bytes, hipDevice_t d) {
  init();
  if (!bytes || d < 0 || d >= g_n) return hipErrorInvalidDevice;
  return hsa_amd_memory_pool_get_info(g_dev[d].pool, HSA_AMD_MEMORY_POOL_INFO_SIZE, bytes) == HSA_STATUS_SUCCESS
             ? hipSuccess : hipErrorInvalidValue;
}

hipError_t hipDeviceCanAccessPeer(int* can, int d, int peer) {
  init();
  if (!can || d < 0 || d >= g_n || peer < 0 || peer >= g_n) return hipErrorInvalidDevice;
  *can = d != peer;
  return hipSuccess;
}

hipError_t hipDeviceEnablePeerAccess(int peer, unsigned int) {
  init();
  if (peer < 0 || peer >= g_n || peer == t_dev) return hipErrorInvalidDevice;  // CLR: not itself
  return hipSuccess;
}

hipError_t hipStreamGetDevice(hipStream_t stream, hipDevice_t* device) {
  init();
  if (!device) return hipErrorInvalidValue;
  *device = dev_of(stream);
  return hipSuccess;
}

hipError_t hipStreamCreate(hipStream_t* stream) {
  init();
  FakeStream* s = new FakeStream{nullptr, t_dev};
  if (hsa_queue_create(g_dev[t_dev].agent, 4096, HSA_QUEUE_TYPE_MULTI, nullptr, nullptr, 0, 0, &s->q) !=
      HSA_STATUS_SUCCESS) {
    delete s;
    return hipErrorOutOfMemory;
  }
  *stream = reinterpret_cast<hipStream_t>(s);
  return hipSuccess;
}

hipError_t hipStreamDestroy(hipStream_t stream) {
  FakeStream* s = reinterpret_cast<FakeStream*>(stream);
  hsa_queue_destroy(s->q);
  delete s;
  return hipSuccess;
}


hipError_t hipLaunchKernel(const void* function_address, dim3, dim3, void**, size_t, hipStream_t stream) {
  init();
  fake_hip_record("hipLaunchKernel");
  if (!function_address) return hipErrorInvalidValue;
  submit(dev_of(stream), *static_cast<const uint32_t*>(function_address), queue_of(stream));
  return hipSuccess;
}

hipError_t hipGraphLaunch(hipGraphExec_t graphExec, hipStream_t stream) {
  init();
  fake_hip_record("hipGraphLaunch");
  if (!graphExec) return hipErrorInvalidValue;
  submit(dev_of(stream), *reinterpret_cast<const uint32_t*>(graphExec), queue_of(stream));
  return hipSuccess;
}

hipError_t hipDeviceSynchronize() {
  init();
  Device& D = g_dev[t_dev];
  std::unique_lock<std::mutex> l(D.mu);
  D.cv.wait(l, [&] { return D.work.empty(); });
  return hipSuccess;
}

hipError_t hipStreamSynchronize(hipStream_t stream) {
  int d = dev_of(stream);
  Device& D = g_dev[d];
  std::unique_lock<std::mutex> l(D.mu);
  D.cv.wait(l, [&] { return D.work.empty(); });
  return hipSuccess;
}

// Every generated stand-in (fake_hip_gates.cpp) records its name: the harness checks that
// a gated call reached the runtime.
static std::mutex g_rec_mu;
static std::string g_last_call;
void fake_hip_record(const char* name) {
  std::lock_guard<std::mutex> l(g_rec_mu);
  g_last_call = name;
}
const char* fake_hip_last_call() {
  static thread_local std::string copy;
  std::lock_guard<std::mutex> l(g_rec_mu);
  copy = g_last_call;
  return copy.c_str();
}

// Entry-point lookup by name, as CLR answers it (the runtime's own definition). The
// library is found from a file-local anchor: the address of an exported function would
// be the preloaded shim's.
static void fake_anchor() {}

hipError_t hipGetProcAddress(const char* symbol, void** pfn, int, uint64_t, hipDriverProcAddressQueryResult* st) {
  Dl_info self;
  void* p = nullptr;
  if (dladdr(reinterpret_cast<void*>(&fake_anchor), &self)) {
    if (void* h = dlopen(self.dli_fname, RTLD_NOLOAD | RTLD_LAZY)) {
      p = dlsym(h, symbol);
      dlclose(h);
    }
  }
  if (st) *st = p ? HIP_GET_PROC_ADDRESS_SUCCESS : HIP_GET_PROC_ADDRESS_SYMBOL_NOT_FOUND;
  if (pfn) *pfn = p;
  return p ? hipSuccess : hipErrorNotFound;
}

// Pinned host memory: a CPU-pool allocation, or a lock of the caller's range (as in CLR).
hipError_t hipHostMalloc(void** ptr, size_t size, unsigned int) {
  init();
  fake_hip_record("hipHostMalloc");
  if (!ptr) return hipErrorInvalidValue;
  return hsa_amd_memory_pool_allocate(g_cpu_pool, size ? size : 1, 0, ptr) == HSA_STATUS_SUCCESS ? hipSuccess
                                                                                                 : hipErrorOutOfMemory;
}

hipError_t hipHostFree(void* ptr) {
  fake_hip_record("hipHostFree");
  if (!ptr) return hipSuccess;
  return hsa_amd_memory_pool_free(ptr) == HSA_STATUS_SUCCESS ? hipSuccess : hipErrorInvalidValue;
}

hipError_t hipHostRegister(void* ptr, size_t size, unsigned int) {
  init();
  fake_hip_record("hipHostRegister");
  if (!ptr || !size) return hipErrorInvalidValue;
  void* agent_ptr = nullptr;
  hsa_status_t st = hsa_amd_memory_lock_to_pool(ptr, size, g_nall ? g_all : nullptr, g_nall, g_cpu_pool, 0, &agent_ptr);
  return st == HSA_STATUS_SUCCESS ? hipSuccess : hipErrorOutOfMemory;
}

hipError_t hipHostUnregister(void* ptr) {
  fake_hip_record("hipHostUnregister");
  if (!ptr) return hipErrorInvalidValue;
  return hsa_amd_memory_unlock(ptr) == HSA_STATUS_SUCCESS ? hipSuccess : hipErrorHostMemoryNotRegistered;
}

// System-allocated memory placed with SVM attributes, as CLR does for hipMemAdvise /
// hipMemPrefetchAsync on memory it did not allocate (device -1 = the CPU).
hsa_agent_t placement_agent(int device) {
  if (device >= 0 && device < g_n) return g_dev[device].agent;
  return device == hipCpuDeviceId ? g_cpu : hsa_agent_t{0};
}

hipError_t hipMemPrefetchAsync(const void* ptr, size_t count, int device, hipStream_t) {
  init();
  fake_hip_record("hipMemPrefetchAsync");
  hsa_agent_t a = placement_agent(device);
  if (!ptr || !count || !a.handle) return hipErrorInvalidValue;
  hsa_signal_t sig;
  hsa_signal_create(1, 0, nullptr, &sig);
  hsa_status_t st = hsa_amd_svm_prefetch_async(const_cast<void*>(ptr), count, a, 0, nullptr, sig);
  hsa_signal_destroy(sig);
  return st == HSA_STATUS_SUCCESS ? hipSuccess
         : st == HSA_STATUS_ERROR_OUT_OF_RESOURCES ? hipErrorOutOfMemory : hipErrorInvalidValue;
}

hipError_t hipMemAdvise(const void* ptr, size_t count, hipMemoryAdvise advice, int device) {
  init();
  fake_hip_record("hipMemAdvise");
  hsa_agent_t a = placement_agent(device);
  if (!ptr || !count || !a.handle) return hipErrorInvalidValue;
  hsa_amd_svm_attribute_pair_t attr{HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION, a.handle};
  if (advice == hipMemAdviseSetAccessedBy) attr = {HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE, a.handle};
  else if (advice != hipMemAdviseSetPreferredLocation) return hipSuccess;
  hsa_status_t st = hsa_amd_svm_attributes_set(const_cast<void*>(ptr), count, &attr, 1);
  return st == HSA_STATUS_SUCCESS ? hipSuccess
         : st == HSA_STATUS_ERROR_OUT_OF_RESOURCES ? hipErrorOutOfMemory : hipErrorInvalidValue;
}

// Test introspection: GPU time executed on `dev` so far, and its kernel count.
uint64_t fake_hip_busy_us(int dev, uint64_t* kernels) {
  if (dev < 0 || dev >= g_n) return 0;
  std::lock_guard<std::mutex> l(g_dev[dev].mu);
  if (kernels) *kernels = g_dev[dev].kernels;
  return g_dev[dev].busy_us;
}

hsa_queue_t* fake_hip_stream_queue(hipStream_t stream) { return reinterpret_cast<FakeStream*>(stream)->q; }

// The CU count as CLR sees it (hipDeviceProp multiProcessorCount): the agent query goes
// through the preloaded shim like the real runtime's.
int fake_hip_device_cus(int dev) {
  init();
  if (dev < 0 || dev >= g_n) return -1;
  uint32_t v = 0;
  hsa_agent_get_info(g_dev[dev].agent, (hsa_agent_info_t)HSA_AMD_AGENT_INFO_COOPERATIVE_COMPUTE_UNIT_COUNT, &v);
  return (int)v;
}

}  // extern "C"
