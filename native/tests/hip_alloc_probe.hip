// Allocation probe linked against libamdhip64 the normal way (global symbol scope), so
// every HIP call goes through the preloaded shim exactly like a C++/HIP application's
// would (ctypes lookups with a library handle would bypass the interposer).
//   hip_alloc_probe managed   hipMallocManaged 1.5 GiB, 1 GiB, free, 1 GiB  -> JSON rcs
//   hip_alloc_probe malloc    hipMalloc the same sequence                   -> JSON rcs
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

int main(int argc, char** argv) {
  bool managed = argc > 1 && !strcmp(argv[1], "managed");
  void *a = nullptr, *b = nullptr, *d = nullptr;
  auto alloc = [&](void** p, size_t n) -> int {
    return managed ? (int)hipMallocManaged(p, n, hipMemAttachGlobal) : (int)hipMalloc(p, n);
  };
  int r1 = alloc(&a, 1536ull << 20);
  int r2 = alloc(&b, 1024ull << 20);
  int f1 = (int)hipFree(a);
  int r3 = alloc(&d, 1024ull << 20);
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  printf("{\"r1\": %d, \"r2\": %d, \"f1\": %d, \"r3\": %d, \"free\": %zu, \"total\": %zu}\n", r1, r2, f1, r3, free_b,
         total_b);
  if (b) (void)hipFree(b);
  if (d) (void)hipFree(d);
  return 0;
}
