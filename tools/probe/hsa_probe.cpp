// Diagnostic interposer: logs which ROCr entry points HIP uses for allocation,
// memory-info queries and queue creation. Used once to validate the shim design
// (SURVEY.md §7.1 "verify on box") — not part of the product.
#include <dlfcn.h>
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <atomic>
#include <cstdio>
#include <cstdlib>

#include <link.h>
#include <cstring>
static void* hsa_handle() {
  static void* h = nullptr;
  if (h) return h;
  dl_iterate_phdr([](struct dl_phdr_info* info, size_t, void*) -> int {
    if (info->dlpi_name && strstr(info->dlpi_name, "libhsa-runtime64.so")) {
      h = dlopen(info->dlpi_name, RTLD_NOLOAD | RTLD_LAZY);
      return h ? 1 : 0;
    }
    return 0;
  }, nullptr);
  return h;
}
static void* real_sym(const char* n) {
  void* p = nullptr;
  if (void* h = hsa_handle()) p = dlvsym(h, n, "ROCR_1");
  if (!p) p = dlvsym(RTLD_NEXT, n, "ROCR_1");
  if (!p) { fprintf(stderr, "[probe] cannot resolve %s\n", n); abort(); }
  return p;
}
#define REAL(name) static auto real = reinterpret_cast<decltype(&name)>(real_sym(#name));

static std::atomic<long> n_alloc{0}, n_free{0}, n_pinfo{0}, n_ainfo{0}, n_q{0}, n_mask{0}, n_vmem{0};

extern "C" {
hsa_status_t hsa_amd_memory_pool_allocate(hsa_amd_memory_pool_t pool, size_t size, uint32_t flags, void** ptr) {
  REAL(hsa_amd_memory_pool_allocate);
  hsa_status_t s = real(pool, size, flags, ptr);
  long n = ++n_alloc;
  if (n < 40 || size > (64u << 20)) fprintf(stderr, "[probe] pool_allocate pool=%lx size=%zu flags=%u -> %p st=%d\n", (long)pool.handle, size, flags, ptr ? *ptr : nullptr, s);
  return s;
}
hsa_status_t hsa_amd_memory_pool_free(void* ptr) {
  REAL(hsa_amd_memory_pool_free);
  ++n_free;
  return real(ptr);
}
hsa_status_t hsa_amd_memory_pool_get_info(hsa_amd_memory_pool_t pool, hsa_amd_memory_pool_info_t attr, void* value) {
  REAL(hsa_amd_memory_pool_get_info);
  hsa_status_t s = real(pool, attr, value);
  ++n_pinfo;
  if (attr == HSA_AMD_MEMORY_POOL_INFO_SIZE) fprintf(stderr, "[probe] pool_get_info SIZE pool=%lx -> %zu\n", (long)pool.handle, *(size_t*)value);
  return s;
}
hsa_status_t hsa_agent_get_info(hsa_agent_t agent, hsa_agent_info_t attr, void* value) {
  REAL(hsa_agent_get_info);
  hsa_status_t s = real(agent, attr, value);
  ++n_ainfo;
  if ((int)attr == HSA_AMD_AGENT_INFO_MEMORY_AVAIL) fprintf(stderr, "[probe] agent_get_info MEMORY_AVAIL agent=%lx -> %lu\n", (long)agent.handle, *(uint64_t*)value);
  if ((int)attr == HSA_AMD_AGENT_INFO_COMPUTE_UNIT_COUNT) fprintf(stderr, "[probe] agent_get_info CU_COUNT -> %u\n", *(uint32_t*)value);
  return s;
}
hsa_status_t hsa_queue_create(hsa_agent_t agent, uint32_t size, hsa_queue_type32_t type,
                              void (*cb)(hsa_status_t, hsa_queue_t*, void*), void* data,
                              uint32_t priv, uint32_t group, hsa_queue_t** queue) {
  REAL(hsa_queue_create);
  hsa_status_t s = real(agent, size, type, cb, data, priv, group, queue);
  ++n_q;
  fprintf(stderr, "[probe] queue_create agent=%lx size=%u -> st=%d q=%p\n", (long)agent.handle, size, s, queue ? (void*)*queue : nullptr);
  if (s == HSA_STATUS_SUCCESS && getenv("PROBE_CU_MASK")) {
    static auto setm = reinterpret_cast<decltype(&hsa_amd_queue_cu_set_mask)>(real_sym("hsa_amd_queue_cu_set_mask"));
    uint32_t m[8] = {0};
    unsigned ncu = (unsigned)atoi(getenv("PROBE_CU_MASK"));
    for (unsigned i = 0; i < ncu && i < 256; i++) m[i / 32] |= 1u << (i % 32);
    hsa_status_t ms = setm(*queue, 256, m);
    fprintf(stderr, "[probe] applied cu mask first %u CUs st=%d\n", ncu, ms);
  }
  return s;
}
hsa_status_t hsa_amd_queue_cu_set_mask(const hsa_queue_t* q, uint32_t n, const uint32_t* m) {
  REAL(hsa_amd_queue_cu_set_mask);
  ++n_mask;
  fprintf(stderr, "[probe] user cu_set_mask n=%u\n", n);
  return real(q, n, m);
}
hsa_status_t hsa_amd_vmem_handle_create(hsa_amd_memory_pool_t pool, size_t size, hsa_amd_memory_type_t type,
                                        uint64_t flags, hsa_amd_vmem_alloc_handle_t* h) {
  REAL(hsa_amd_vmem_handle_create);
  ++n_vmem;
  fprintf(stderr, "[probe] vmem_handle_create size=%zu\n", size);
  return real(pool, size, type, flags, h);
}
}

__attribute__((destructor)) static void fini() {
  fprintf(stderr, "[probe] totals alloc=%ld free=%ld pool_info=%ld agent_info=%ld queues=%ld user_masks=%ld vmem=%ld\n",
          n_alloc.load(), n_free.load(), n_pinfo.load(), n_ainfo.load(), n_q.load(), n_mask.load(), n_vmem.load());
}
