// A fake ROCr (libhsa-runtime64.so.1) for testing the interception shim on a CPU-only
// machine: N GPU agents with configurable UUIDs, HBM sizes and CU layout, memory pools
// backed by reserved-but-never-touched address space, queues that record the CU masks
// and priorities applied to them, and a fake KFD process tree (vram_<gpu_id>,
// stats_<gpu_id>/cu_occupancy) under $FAKE_KFD_ROOT for the process's fake host PID
// (getpid() + $FAKE_KFD_PID_OFFSET, so the shim's host-PID discovery has to work as in a
// PID namespace).
//
// Exported with the ROCR_1 symbol version like the real runtime, so the shim's
// interposition and real-symbol resolution (real.cpp) behave exactly as with libamdhip64
// and the real ROCr. Environment:
//   FAKE_ROCR_GPUS      number of GPU agents (default 2)
//   FAKE_ROCR_HBM       bytes of HBM per GPU (default 8 GiB)
//   FAKE_ROCR_CUS / FAKE_ROCR_XCC / FAKE_ROCR_SE   CU layout (256 / 8 / 32 per agent)
//   FAKE_ROCR_UUIDS     comma-separated agent UUIDs (default GPU-fa4e00000000000<i>)
//   FAKE_ROCR_PARTS     agents per PCI address (default 1; 4 = CPX-style compute
//                       partitions exposed as GPUs: consecutive agents share a BDF)
//   FAKE_KFD_ROOT       fake /sys/class/kfd/kfd/proc (unset: no KFD tree)
//   FAKE_KFD_PID_OFFSET host-PID offset (default 100000)
//   FAKE_ROCR_NO_SVM    1: no shared virtual memory (hsa_amd_svm_* refuse, SVM_SUPPORTED false)
//   FAKE_SVM_FAIL       1: every SVM prefetch into a GPU fails (the completion signal goes negative)
//   FAKE_SVM_KFD_VRAM   0: SVM ranges migrated into HBM are not in KFD's vram_<gpu_id> (default 1)
//   FAKE_ROCR_XNACK     1: recoverable page faults reported on (HSA_AMD_SYSTEM_INFO_XNACK_ENABLED)
//   FAKE_SVM_HANG       1: prefetches into a GPU never complete (their signals stay at 1)
//   FAKE_ROCR_SHARED_HBM  file: the GPUs' HBM is shared by every process naming the same
//                       file (a node: several containers' processes on one physical GPU);
//                       admission and MEMORY_AVAIL then see every process's usage
//   FAKE_SVM_AVAIL_BLIND  1: MEMORY_AVAIL does not count SVM pages migrated into HBM (as ROCr
//                       on MI355X, profiles/r4b); admission still does (the VRAM is taken)
// Test-only introspection: fake_rocr_* functions below.
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <errno.h>
#include <pthread.h>
#include <fcntl.h>
#include <sys/mman.h>
#include <sys/stat.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <map>
#include <mutex>
#include <string>
#include <vector>

namespace {

constexpr uint64_t kCpuAgent = 100;
constexpr uint64_t kGpuPoolBase = 1000;
constexpr uint64_t kCpuPool = 2000;

struct FakeGpu {
  std::string uuid;
  uint64_t hbm = 8ull << 30;
  std::atomic<uint64_t> used{0};     // this process's bytes in HBM (SVM included)
  std::atomic<uint64_t> svm_used{0};  // of which SVM pages
  uint32_t gpu_id = 0;
};

// Node-wide HBM of each GPU (FAKE_ROCR_SHARED_HBM): bytes in use by every process, and of
// them SVM pages.
struct SharedHbm {
  std::atomic<uint64_t> used[16];
  std::atomic<uint64_t> svm[16];
};

struct FakeQueue {
  hsa_queue_t q;
  std::atomic<uint64_t> wr{0}, rd{0};  // AQL write / read dispatch indices (fake_hip moves them)
  int dev;
  uint32_t mask[8];
  int mask_bits;
  int mask_sets;
  int priority;
};

// An SVM range: the application's own host memory registered for GPU access. Its pages are
// real memory (the caller's mapping), so data survives a "migration", which only moves the
// range's location and its bytes in and out of the GPU's HBM.
struct SvmRange {
  uint64_t size = 0;
  std::map<uint64_t, uint64_t> access;  // agent -> access attribute
  uint64_t pref = 0, loc = 0;           // preferred / current location (agent handle, 0 = host)
};

struct State {
  int n = 2;
  int cus = 256, xcc = 8, se = 32, parts = 1;
  FakeGpu gpus[16];
  std::mutex mu;
  std::map<uintptr_t, std::pair<int, uint64_t>> allocs;  // ptr -> (dev or -1 for host, size)
  std::map<uintptr_t, FakeQueue*> queues;
  std::map<uintptr_t, SvmRange> svm;
  std::map<uintptr_t, int> locks;  // locked host ranges -> lock count
  char* arena = nullptr;
  uint64_t arena_size = 0, arena_next = 0;
  std::string kfd;  // fake KFD process dir of this process ("" = none)
  SharedHbm* node = nullptr;  // FAKE_ROCR_SHARED_HBM (null: this process's HBM is its own)
  bool inited = false;
  int init_count = 0;
};

State& st() {
  static State* s = new State();
  return *s;
}

uint64_t env_u64(const char* k, uint64_t d) {
  const char* v = getenv(k);
  return v && *v ? strtoull(v, nullptr, 0) : d;
}

void write_file(const std::string& path, uint64_t v) {
  FILE* f = fopen(path.c_str(), "w");
  if (!f) return;
  fprintf(f, "%llu\n", (unsigned long long)v);
  fclose(f);
}

// HBM bytes in use on GPU `d` as the driver sees them (every process on a shared node).
uint64_t hbm_used(int d) {
  State& s = st();
  return s.node ? s.node->used[d].load() : s.gpus[d].used.load();
}

// MEMORY_AVAIL's view: without the SVM pages when FAKE_SVM_AVAIL_BLIND=1.
uint64_t hbm_used_avail(int d) {
  State& s = st();
  const bool blind = env_u64("FAKE_SVM_AVAIL_BLIND", 0) != 0;
  const uint64_t u = hbm_used(d);
  const uint64_t v = blind ? (s.node ? s.node->svm[d].load() : s.gpus[d].svm_used.load()) : 0;
  return u > v ? u - v : 0;
}

void add_used(int d, int64_t delta, bool svm) {
  State& s = st();
  s.gpus[d].used.fetch_add((uint64_t)delta);
  if (svm) s.gpus[d].svm_used.fetch_add((uint64_t)delta);
  if (s.node) {
    s.node->used[d].fetch_add((uint64_t)delta);
    if (svm) s.node->svm[d].fetch_add((uint64_t)delta);
  }
}

void kfd_update_vram(int dev) {
  State& s = st();
  if (s.kfd.empty() || dev < 0) return;
  const uint64_t svm = env_u64("FAKE_SVM_KFD_VRAM", 1) ? 0 : s.gpus[dev].svm_used.load();
  write_file(s.kfd + "/vram_" + std::to_string(s.gpus[dev].gpu_id), s.gpus[dev].used.load() - svm);
}

// A forked child is a new KFD process: its own (empty) process directory and no HBM of its
// own - what the driver gives a child that opens the GPU, so the shim's host-PID discovery in
// the child finds the child, not the parent.
void fake_atfork_child() {
  State& s = st();
  if (!s.inited || s.kfd.empty()) return;
  const char* root = getenv("FAKE_KFD_ROOT");
  if (!root) return;
  s.kfd = std::string(root) + "/" + std::to_string((int)getpid() + (int)env_u64("FAKE_KFD_PID_OFFSET", 100000));
  mkdir(s.kfd.c_str(), 0777);
  for (int i = 0; i < s.n; i++) {
    s.gpus[i].used.store(0);
    s.gpus[i].svm_used.store(0);
    std::string stats = s.kfd + "/stats_" + std::to_string(s.gpus[i].gpu_id);
    mkdir(stats.c_str(), 0777);
    write_file(stats + "/cu_occupancy", 0);
    kfd_update_vram(i);
  }
}

void setup() {
  State& s = st();
  if (s.inited) return;
  pthread_atfork(nullptr, nullptr, fake_atfork_child);
  s.n = (int)env_u64("FAKE_ROCR_GPUS", 2);
  if (s.n < 1) s.n = 1;
  if (s.n > 16) s.n = 16;
  s.cus = (int)env_u64("FAKE_ROCR_CUS", 256);
  s.parts = (int)env_u64("FAKE_ROCR_PARTS", 1);
  if (s.parts < 1) s.parts = 1;
  s.xcc = (int)env_u64("FAKE_ROCR_XCC", 8);
  s.se = (int)env_u64("FAKE_ROCR_SE", 32);
  uint64_t hbm = env_u64("FAKE_ROCR_HBM", 8ull << 30);
  std::vector<std::string> uuids;
  if (const char* u = getenv("FAKE_ROCR_UUIDS")) {
    std::string all(u);
    size_t p = 0;
    while (p <= all.size()) {
      size_t c = all.find(',', p);
      if (c == std::string::npos) c = all.size();
      if (c > p) uuids.push_back(all.substr(p, c - p));
      p = c + 1;
    }
  }
  for (int i = 0; i < s.n; i++) {
    char buf[64];
    snprintf(buf, sizeof(buf), "GPU-fa4e%012x", i);
    s.gpus[i].uuid = i < (int)uuids.size() ? uuids[i] : buf;
    s.gpus[i].hbm = hbm;
    s.gpus[i].gpu_id = 1000 + i;
  }
  if (const char* path = getenv("FAKE_ROCR_SHARED_HBM")) {
    int fd = open(path, O_RDWR | O_CREAT, 0666);
    if (fd >= 0) {
      if (ftruncate(fd, sizeof(SharedHbm)) == 0) {
        void* m = mmap(nullptr, sizeof(SharedHbm), PROT_READ | PROT_WRITE, MAP_SHARED, fd, 0);
        if (m != MAP_FAILED) s.node = static_cast<SharedHbm*>(m);
      }
      close(fd);
    }
  }
  s.arena_size = 1ull << 42;  // 4 TiB of address space, never touched
  void* p = mmap(nullptr, s.arena_size, PROT_NONE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  s.arena = p == MAP_FAILED ? nullptr : static_cast<char*>(p);
  if (const char* root = getenv("FAKE_KFD_ROOT")) {
    int hp = (int)getpid() + (int)env_u64("FAKE_KFD_PID_OFFSET", 100000);
    s.kfd = std::string(root) + "/" + std::to_string(hp);
    mkdir(root, 0777);
    mkdir(s.kfd.c_str(), 0777);
    for (int i = 0; i < s.n; i++) {
      std::string stats = s.kfd + "/stats_" + std::to_string(s.gpus[i].gpu_id);
      mkdir(stats.c_str(), 0777);
      write_file(stats + "/cu_occupancy", 0);
      kfd_update_vram(i);
    }
  }
  s.inited = true;
}

int gpu_of(hsa_agent_t a) {
  if (a.handle >= 1 && a.handle <= (uint64_t)st().n) return (int)a.handle - 1;
  return -1;
}

void* bump(uint64_t size) {
  State& s = st();
  uint64_t sz = (size + 0xFFFF) & ~0xFFFFull;
  if (!s.arena || s.arena_next + sz > s.arena_size) return nullptr;
  void* p = s.arena + s.arena_next;
  s.arena_next += sz + 0x10000;  // guard gap
  return p;
}

bool svm_on() { return !env_u64("FAKE_ROCR_NO_SVM", 0); }

// Drops SVM ranges whose memory the application unmapped (KFD learns of it through its MMU
// notifier): a range in HBM gives its bytes back. Caller holds the state lock.
void svm_gc() {
  State& s = st();
  const long pg = sysconf(_SC_PAGESIZE);
  for (auto it = s.svm.begin(); it != s.svm.end();) {
    unsigned char v;
    if (mincore(reinterpret_cast<void*>(it->first), (size_t)pg, &v) != 0 && errno == ENOMEM) {
      const int d = gpu_of(hsa_agent_t{it->second.loc});
      if (d >= 0) {
        add_used(d, -(int64_t)it->second.size, true);
        if (env_u64("FAKE_SVM_KFD_VRAM", 1)) kfd_update_vram(d);
      }
      it = s.svm.erase(it);
    } else {
      ++it;
    }
  }
}

}  // namespace

extern "C" {

hsa_status_t hsa_init() {
  std::lock_guard<std::mutex> g(st().mu);
  setup();
  st().init_count++;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_shut_down() { return HSA_STATUS_SUCCESS; }

hsa_status_t hsa_iterate_agents(hsa_status_t (*cb)(hsa_agent_t, void*), void* data) {
  setup();
  hsa_status_t r = cb(hsa_agent_t{kCpuAgent}, data);
  if (r != HSA_STATUS_SUCCESS) return r;
  for (int i = 0; i < st().n; i++) {
    r = cb(hsa_agent_t{(uint64_t)i + 1}, data);
    if (r != HSA_STATUS_SUCCESS) return r;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  setup();
  State& s = st();
  int d = gpu_of(agent);
  if ((int)attr == HSA_AGENT_INFO_DEVICE) {
    *static_cast<hsa_device_type_t*>(value) = d >= 0 ? HSA_DEVICE_TYPE_GPU : HSA_DEVICE_TYPE_CPU;
    return HSA_STATUS_SUCCESS;
  }
  if (d < 0) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  switch ((int)attr) {
    case HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT: *static_cast<uint32_t*>(value) = s.cus; break;
    case HSA_AMD_AGENT_INFO_COOPERATIVE_COMPUTE_UNIT_COUNT: *static_cast<uint32_t*>(value) = s.cus; break;
    case HSA_AMD_AGENT_INFO_NUM_XCC: *static_cast<uint32_t*>(value) = s.xcc; break;
    case HSA_AMD_AGENT_INFO_NUM_SHADER_ENGINES: *static_cast<uint32_t*>(value) = s.se; break;
    case HSA_AMD_AGENT_INFO_DRIVER_UID: *static_cast<uint32_t*>(value) = s.gpus[d].gpu_id; break;
    case HSA_AMD_AGENT_INFO_MAX_WAVES_PER_CU: *static_cast<uint32_t*>(value) = 32; break;
    case HSA_AMD_AGENT_INFO_NEAREST_CPU: *static_cast<hsa_agent_t*>(value) = hsa_agent_t{kCpuAgent}; break;
    case HSA_AMD_AGENT_INFO_UUID: snprintf(static_cast<char*>(value), 64, "%s", s.gpus[d].uuid.c_str()); break;
    case HSA_AMD_AGENT_INFO_BDFID: *static_cast<uint32_t*>(value) = (uint32_t)(0x05 + 0x10 * (d / s.parts)) << 8; break;
    case HSA_AMD_AGENT_INFO_DOMAIN: *static_cast<uint32_t*>(value) = 0; break;
    case HSA_AMD_AGENT_INFO_MEMORY_AVAIL: {
      {
        std::lock_guard<std::mutex> g(s.mu);
        svm_gc();
      }
      uint64_t u = hbm_used_avail(d);
      *static_cast<uint64_t*>(value) = s.gpus[d].hbm > u ? s.gpus[d].hbm - u : 0;
      break;
    }
    default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_agent_iterate_memory_pools(hsa_agent_t agent,
                                                hsa_status_t (*cb)(hsa_amd_memory_pool_t, void*), void* data) {
  int d = gpu_of(agent);
  if (agent.handle == kCpuAgent) return cb(hsa_amd_memory_pool_t{kCpuPool}, data);
  if (d < 0) return HSA_STATUS_ERROR_INVALID_AGENT;
  return cb(hsa_amd_memory_pool_t{kGpuPoolBase + (uint64_t)d}, data);
}

hsa_status_t hsa_amd_memory_pool_get_info(hsa_amd_memory_pool_t pool, hsa_amd_memory_pool_info_t attr, void* value) {
  setup();
  State& s = st();
  int d = pool.handle >= kGpuPoolBase && pool.handle < kGpuPoolBase + (uint64_t)s.n ? (int)(pool.handle - kGpuPoolBase)
                                                                                     : -1;
  if (d < 0 && pool.handle != kCpuPool) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  switch ((int)attr) {
    case HSA_AMD_MEMORY_POOL_INFO_SEGMENT: *static_cast<hsa_amd_segment_t*>(value) = HSA_AMD_SEGMENT_GLOBAL; break;
    case HSA_AMD_MEMORY_POOL_INFO_SIZE: *static_cast<size_t*>(value) = d >= 0 ? s.gpus[d].hbm : (64ull << 30); break;
    case HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS:
      *static_cast<uint32_t*>(value) = HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED;
      break;
    case HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED: *static_cast<bool*>(value) = true; break;
    default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  }
  return HSA_STATUS_SUCCESS;
}

}  // extern "C"

namespace {
// Internal entry points: ROCr's exported functions never call each other through their
// exported symbols (which the preloaded shim interposes), so neither does the fake.
hsa_status_t pool_allocate_impl(hsa_amd_memory_pool_t pool, size_t size, void** ptr) {
  setup();
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  int d = pool.handle >= kGpuPoolBase && pool.handle < kGpuPoolBase + (uint64_t)s.n ? (int)(pool.handle - kGpuPoolBase)
                                                                                     : -1;
  if (d < 0 && pool.handle != kCpuPool) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  if (d >= 0 && hbm_used(d) + size > s.gpus[d].hbm) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  // Host memory is real (the application may touch pinned buffers); HBM is address space only.
  void* p = d >= 0 ? bump(size) : mmap(nullptr, size, PROT_READ | PROT_WRITE, MAP_PRIVATE | MAP_ANONYMOUS | MAP_NORESERVE, -1, 0);
  if (p == MAP_FAILED) p = nullptr;
  if (!p) return HSA_STATUS_ERROR_OUT_OF_RESOURCES;
  s.allocs[reinterpret_cast<uintptr_t>(p)] = {d, size};
  if (d >= 0) {
    add_used(d, (int64_t)size, false);
    kfd_update_vram(d);
  }
  *ptr = p;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t pool_free_impl(void* ptr) {
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  auto it = s.allocs.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == s.allocs.end()) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  int d = it->second.first;
  if (d >= 0) {
    add_used(d, -(int64_t)it->second.second, false);
    kfd_update_vram(d);
  } else {
    munmap(ptr, it->second.second);
  }
  s.allocs.erase(it);
  return HSA_STATUS_SUCCESS;
}
}  // namespace

extern "C" {

hsa_status_t hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t, void** ptr) {
  return pool_allocate_impl(pool, size, ptr);
}
hsa_status_t hsa_amd_memory_pool_free(void* ptr) { return pool_free_impl(ptr); }

// Legacy region API: the GPU's region handle is its pool handle (as in ROCr), and a GPU agent
// also lists the system memory regions it can reach - the CPU pool (ROCr's VisitRegion).
hsa_status_t hsa_agent_iterate_regions(hsa_agent_t agent, hsa_status_t (*cb)(hsa_region_t, void*), void* data) {
  int d = gpu_of(agent);
  if (agent.handle == kCpuAgent) return cb(hsa_region_t{kCpuPool}, data);
  if (d < 0) return HSA_STATUS_ERROR_INVALID_AGENT;
  hsa_status_t r = cb(hsa_region_t{kCpuPool}, data);
  if (r != HSA_STATUS_SUCCESS) return r;
  return cb(hsa_region_t{kGpuPoolBase + (uint64_t)d}, data);
}
hsa_status_t hsa_region_get_info(hsa_region_t region, hsa_region_info_t attr, void* value) {
  if ((int)attr == HSA_REGION_INFO_SEGMENT) {
    *static_cast<hsa_region_segment_t*>(value) = HSA_REGION_SEGMENT_GLOBAL;
    return HSA_STATUS_SUCCESS;
  }
  if ((int)attr == HSA_REGION_INFO_RUNTIME_ALLOC_ALLOWED) {
    *static_cast<bool*>(value) = true;
    return HSA_STATUS_SUCCESS;
  }
  if ((int)attr == HSA_REGION_INFO_GLOBAL_FLAGS) {
    *static_cast<uint32_t*>(value) = HSA_REGION_GLOBAL_FLAG_COARSE_GRAINED;
    return HSA_STATUS_SUCCESS;
  }
  return HSA_STATUS_ERROR_INVALID_ARGUMENT;
}
hsa_status_t hsa_memory_allocate(hsa_region_t region, size_t size, void** ptr) {
  return pool_allocate_impl(hsa_amd_memory_pool_t{region.handle}, size, ptr);
}
hsa_status_t hsa_memory_free(void* ptr) { return pool_free_impl(ptr); }

// Memory locks: a locked user range, counted per address (test introspection: fake_rocr_locked).
static hsa_status_t lock_impl(void* host_ptr, size_t size, void** agent_ptr) {
  if (!host_ptr || !size) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  std::lock_guard<std::mutex> g(st().mu);
  st().locks[reinterpret_cast<uintptr_t>(host_ptr)]++;
  if (agent_ptr) *agent_ptr = host_ptr;
  return HSA_STATUS_SUCCESS;
}
hsa_status_t hsa_amd_memory_lock(void* host_ptr, size_t size, hsa_agent_t*, int, void** agent_ptr) {
  return lock_impl(host_ptr, size, agent_ptr);
}
hsa_status_t hsa_amd_memory_lock_to_pool(void* host_ptr, size_t size, hsa_agent_t*, int, hsa_amd_memory_pool_t,
                                         uint32_t, void** agent_ptr) {
  return lock_impl(host_ptr, size, agent_ptr);
}
hsa_status_t hsa_amd_memory_unlock(void* host_ptr) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().locks.find(reinterpret_cast<uintptr_t>(host_ptr));
  if (it == st().locks.end()) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  if (--it->second == 0) st().locks.erase(it);
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_agents_allow_access(uint32_t, const hsa_agent_t*, const uint32_t*, const void*) {
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                              void (*)(hsa_status_t, hsa_queue_t*, void*), void*, uint32_t, uint32_t,
                              hsa_queue_t** queue) {
  int d = gpu_of(agent);
  if (d < 0) return HSA_STATUS_ERROR_INVALID_AGENT;
  FakeQueue* q = new FakeQueue();
  memset(&q->q, 0, sizeof(q->q));
  q->q.type = type;
  q->q.size = size;
  q->dev = d;
  memset(q->mask, 0xff, sizeof(q->mask));
  q->mask_bits = st().cus;
  q->mask_sets = 0;
  q->priority = 1;
  std::lock_guard<std::mutex> g(st().mu);
  st().queues[reinterpret_cast<uintptr_t>(&q->q)] = q;
  *queue = &q->q;
  return HSA_STATUS_SUCCESS;
}

// The queue's dispatch indices: fake_hip submits (write index) and retires (read index)
// the kernels it runs on a stream's queue, as the CP would.
uint64_t hsa_queue_load_write_index_relaxed(const hsa_queue_t* queue) {
  return reinterpret_cast<const FakeQueue*>(queue)->wr.load();
}
uint64_t hsa_queue_load_read_index_relaxed(const hsa_queue_t* queue) {
  return reinterpret_cast<const FakeQueue*>(queue)->rd.load();
}
void fake_rocr_queue_submit(hsa_queue_t* queue) { reinterpret_cast<FakeQueue*>(queue)->wr.fetch_add(1); }
void fake_rocr_queue_retire(hsa_queue_t* queue) { reinterpret_cast<FakeQueue*>(queue)->rd.fetch_add(1); }

hsa_status_t hsa_queue_destroy(hsa_queue_t* queue) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().queues.find(reinterpret_cast<uintptr_t>(queue));
  if (it == st().queues.end()) return HSA_STATUS_ERROR_INVALID_QUEUE;
  delete it->second;
  st().queues.erase(it);
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* queue, uint32_t num_cu_mask_count, const uint32_t* cu_mask) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().queues.find(reinterpret_cast<uintptr_t>(queue));
  if (it == st().queues.end()) return HSA_STATUS_ERROR_INVALID_QUEUE;
  FakeQueue* q = it->second;
  memset(q->mask, 0, sizeof(q->mask));
  for (uint32_t i = 0; i < num_cu_mask_count && i < 256; i++)
    if ((cu_mask[i / 32] >> (i % 32)) & 1u) q->mask[i / 32] |= 1u << (i % 32);
  q->mask_bits = (int)num_cu_mask_count;
  q->mask_sets++;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_queue_set_priority(hsa_queue_t* queue, hsa_amd_queue_priority_t priority) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().queues.find(reinterpret_cast<uintptr_t>(queue));
  if (it == st().queues.end()) return HSA_STATUS_ERROR_INVALID_QUEUE;
  it->second->priority = (int)priority;
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_vmem_handle_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t, uint64_t,
                                        hsa_amd_vmem_alloc_handle_t* handle) {
  void* p = nullptr;
  hsa_status_t r = pool_allocate_impl(pool, size, &p);
  if (r == HSA_STATUS_SUCCESS) handle->handle = reinterpret_cast<uint64_t>(p);
  return r;
}

hsa_status_t hsa_amd_vmem_handle_release(hsa_amd_vmem_alloc_handle_t handle) {
  return pool_free_impl(reinterpret_cast<void*>(handle.handle));
}

// IPC export works on device memory only, as measured on MI355X (profiles/r5e): a GPU-pool
// allocation exports; a system-pool allocation (pinned host memory) and ordinary memory
// registered as an SVM range do not.
// len 0 = the whole allocation (the fake HIP's hipIpcGetMemHandle does not know the size).
hsa_status_t hsa_amd_ipc_memory_create(void* ptr, size_t len, hsa_amd_ipc_memory_t* handle) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().allocs.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == st().allocs.end() || it->second.first < 0 || (len && len != it->second.second))
    return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  if (handle) {
    memset(handle, 0, sizeof(*handle));
    memcpy(handle, &it->first, sizeof(it->first));
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_ipc_memory_attach(const hsa_amd_ipc_memory_t*, size_t len, uint32_t, const hsa_agent_t*,
                                       void** mapped_ptr) {
  std::lock_guard<std::mutex> g(st().mu);
  *mapped_ptr = bump(len);
  return *mapped_ptr ? HSA_STATUS_SUCCESS : HSA_STATUS_ERROR_OUT_OF_RESOURCES;
}

hsa_status_t hsa_amd_ipc_memory_detach(void*) { return HSA_STATUS_SUCCESS; }

hsa_status_t hsa_system_get_info(hsa_system_info_t attr, void* value) {
  switch ((int)attr) {
    case HSA_AMD_SYSTEM_INFO_SVM_SUPPORTED: *static_cast<bool*>(value) = svm_on(); return HSA_STATUS_SUCCESS;
    case HSA_AMD_SYSTEM_INFO_SVM_ACCESSIBLE_BY_DEFAULT: *static_cast<bool*>(value) = false; return HSA_STATUS_SUCCESS;
    case HSA_AMD_SYSTEM_INFO_XNACK_ENABLED: *static_cast<bool*>(value) = env_u64("FAKE_ROCR_XNACK", 0) != 0; return HSA_STATUS_SUCCESS;
    default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  }
}

// Signals: every fake asynchronous operation completes before it returns, so a wait only
// reads the value.
hsa_status_t hsa_signal_create(hsa_signal_value_t initial, uint32_t, const hsa_agent_t*, hsa_signal_t* sig) {
  sig->handle = reinterpret_cast<uint64_t>(new std::atomic<int64_t>(initial));
  return HSA_STATUS_SUCCESS;
}
hsa_status_t hsa_signal_destroy(hsa_signal_t sig) {
  delete reinterpret_cast<std::atomic<int64_t>*>(sig.handle);
  return HSA_STATUS_SUCCESS;
}
// A wait spins until the condition holds or the timeout passes (as ROCr's busy wait does).
hsa_signal_value_t hsa_signal_wait_scacquire(hsa_signal_t sig, hsa_signal_condition_t cond, hsa_signal_value_t cmp,
                                             uint64_t timeout, hsa_wait_state_t) {
  auto* a = reinterpret_cast<std::atomic<int64_t>*>(sig.handle);
  const auto t0 = std::chrono::steady_clock::now();
  for (;;) {
    const int64_t v = a->load();
    const bool ok = cond == HSA_SIGNAL_CONDITION_EQ ? v == cmp : cond == HSA_SIGNAL_CONDITION_NE ? v != cmp
                    : cond == HSA_SIGNAL_CONDITION_LT ? v < cmp : v >= cmp;
    if (ok || (uint64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - t0)
                      .count() >= timeout)
      return v;
  }
}
hsa_signal_value_t hsa_signal_load_scacquire(hsa_signal_t sig) {
  return reinterpret_cast<std::atomic<int64_t>*>(sig.handle)->load();
}
void hsa_signal_subtract_screlease(hsa_signal_t sig, hsa_signal_value_t v) {
  reinterpret_cast<std::atomic<int64_t>*>(sig.handle)->fetch_sub(v);
}
void hsa_signal_store_relaxed(hsa_signal_t sig, hsa_signal_value_t v) {
  reinterpret_cast<std::atomic<int64_t>*>(sig.handle)->store(v);
}

hsa_status_t hsa_amd_svm_attributes_set(void* ptr, size_t size, hsa_amd_svm_attribute_pair_t* list, size_t n) {
  if (!svm_on()) return HSA_STATUS_ERROR;
  setup();
  std::lock_guard<std::mutex> g(st().mu);
  svm_gc();
  SvmRange& r = st().svm[reinterpret_cast<uintptr_t>(ptr)];
  r.size = size;
  for (size_t i = 0; i < n; i++) {
    switch (list[i].attribute) {
      case HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE:
      case HSA_AMD_SVM_ATTRIB_AGENT_ACCESSIBLE_IN_PLACE: r.access[list[i].value] = list[i].attribute; break;
      case HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS: r.access.erase(list[i].value); break;
      case HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION: r.pref = list[i].value; break;
      case HSA_AMD_SVM_ATTRIB_GLOBAL_FLAG: case HSA_AMD_SVM_ATTRIB_READ_ONLY: case HSA_AMD_SVM_ATTRIB_GPU_EXEC: break;
      default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
    }
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_svm_attributes_get(void* ptr, size_t, hsa_amd_svm_attribute_pair_t* list, size_t n) {
  if (!svm_on()) return HSA_STATUS_ERROR;
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().svm.find(reinterpret_cast<uintptr_t>(ptr));
  for (size_t i = 0; i < n; i++) {
    switch (list[i].attribute) {
      case HSA_AMD_SVM_ATTRIB_ACCESS_QUERY: {
        uint64_t a = HSA_AMD_SVM_ATTRIB_AGENT_NO_ACCESS;
        if (it != st().svm.end() && it->second.access.count(list[i].value)) a = it->second.access[list[i].value];
        list[i].attribute = a;
        break;
      }
      case HSA_AMD_SVM_ATTRIB_PREFERRED_LOCATION: list[i].value = it != st().svm.end() ? it->second.pref : 0; break;
      case HSA_AMD_SVM_ATTRIB_PREFETCH_LOCATION: list[i].value = it != st().svm.end() ? it->second.loc : 0; break;
      default: return HSA_STATUS_ERROR_INVALID_ARGUMENT;
    }
  }
  return HSA_STATUS_SUCCESS;
}

hsa_status_t hsa_amd_svm_prefetch_async(void* ptr, size_t size, hsa_agent_t agent, uint32_t, const hsa_signal_t*,
                                        hsa_signal_t done) {
  if (!svm_on()) return HSA_STATUS_ERROR;
  State& s = st();
  std::lock_guard<std::mutex> g(s.mu);
  svm_gc();
  auto it = s.svm.find(reinterpret_cast<uintptr_t>(ptr));
  if (it == s.svm.end()) return HSA_STATUS_ERROR_INVALID_ARGUMENT;
  SvmRange& r = it->second;
  auto* sig = reinterpret_cast<std::atomic<int64_t>*>(done.handle);
  const int to = gpu_of(agent), from = gpu_of(hsa_agent_t{r.loc});
  const bool counted = env_u64("FAKE_SVM_KFD_VRAM", 1) != 0;
  if (sig && to >= 0 && env_u64("FAKE_SVM_HANG", 0)) {
    // The migration never completes: the signal stays at its initial value (the caller may not
    // destroy it - the fake's "driver" would still write it); the range does not move.
    return HSA_STATUS_SUCCESS;
  }
  bool ok = to != from || to < 0;
  if (to >= 0 && to != from && (env_u64("FAKE_SVM_FAIL", 0) || hbm_used(to) + size > s.gpus[to].hbm)) ok = false;
  if (ok && to != from) {
    if (from >= 0) {
      add_used(from, -(int64_t)r.size, true);
      if (counted) kfd_update_vram(from);
    }
    if (to >= 0) {
      add_used(to, (int64_t)r.size, true);
      if (counted) kfd_update_vram(to);
    }
    r.loc = to >= 0 ? agent.handle : 0;
  }
  if (sig) {
    if (ok) sig->fetch_sub(1);
    else sig->store(-1);
  }
  return HSA_STATUS_SUCCESS;
}

// ---------------------------------------------------------------- test introspection
// CU mask and priority last applied to `queue`; returns the number of mask changes.
int fake_rocr_queue_state(const hsa_queue_t* queue, uint32_t* mask_words8, int* priority, int* device) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().queues.find(reinterpret_cast<uintptr_t>(queue));
  if (it == st().queues.end()) return -1;
  memcpy(mask_words8, it->second->mask, sizeof(it->second->mask));
  if (priority) *priority = it->second->priority;
  if (device) *device = it->second->dev;
  return it->second->mask_sets;
}

// Bytes the fake runtime holds on GPU `dev` (what a real driver would report).
uint64_t fake_rocr_used(int dev) {
  {
    std::lock_guard<std::mutex> g(st().mu);
    svm_gc();
  }
  return dev >= 0 && dev < st().n ? st().gpus[dev].used.load() : 0;
}

// Whether the SVM range at `ptr` lists `agent` as having access.
int fake_rocr_svm_has_access(const void* ptr, uint64_t agent) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().svm.find(reinterpret_cast<uintptr_t>(ptr));
  return it != st().svm.end() && it->second.access.count(agent) ? 1 : 0;
}

// KFD's MMU notifier: ranges the application unmapped are dropped (with their VRAM) now.
void fake_rocr_svm_gc() {
  std::lock_guard<std::mutex> g(st().mu);
  svm_gc();
}

// Where the SVM range at `ptr` lives: the GPU ordinal, -1 = host memory, -2 = not a range.
int fake_rocr_svm_location(const void* ptr) {
  std::lock_guard<std::mutex> g(st().mu);
  auto it = st().svm.find(reinterpret_cast<uintptr_t>(ptr));
  return it == st().svm.end() ? -2 : gpu_of(hsa_agent_t{it->second.loc});
}

// Memory the runtime allocates internally (scratch, code objects): bypasses every
// allocation entry point, shows up only in KFD's per-process VRAM counter.
int fake_rocr_internal_alloc(int dev, int64_t bytes) {
  if (dev < 0 || dev >= st().n) return -1;
  add_used(dev, bytes, false);
  kfd_update_vram(dev);
  return 0;
}

// Sets the fake cu_occupancy of this process on `dev` (resident waves, CUs' worth).
int fake_rocr_set_occupancy(int dev, int cus) {
  if (st().kfd.empty() || dev < 0 || dev >= st().n) return -1;
  write_file(st().kfd + "/stats_" + std::to_string(st().gpus[dev].gpu_id) + "/cu_occupancy", (uint64_t)cus);
  return 0;
}

int fake_rocr_host_pid() { return (int)getpid() + (int)env_u64("FAKE_KFD_PID_OFFSET", 100000); }

}  // extern "C"
