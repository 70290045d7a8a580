// Allocation probe linked against libamdhip64 the normal way (global symbol scope), so
// every HIP call goes through the preloaded shim exactly like a C++/HIP application's
// would (ctypes lookups with a library handle would bypass the interposer).
//
//   hip_alloc_probe <kind>   allocate 3/4 of the free memory, then 1/2, free the first,
//                            1/2 again -> one JSON line with the return codes and
//                            hipMemGetInfo before and after
//
// kinds (SURVEY.md §7.4 "choke-point completeness": every HIP device allocation API must
// reach the quota):
//   malloc     hipMalloc
//   managed    hipMallocManaged (reference class (a): cuMemAllocManaged)
//   pitch      hipMallocPitch (1 MiB rows; reference cuMemAllocPitch_v2)
//   3d         hipMalloc3D
//   ext        hipExtMallocWithFlags(hipDeviceMallocDefault)
//   async      hipMallocAsync / hipFreeAsync on a stream (default stream-ordered pool,
//              trimmed after the free so the pool returns the memory)
//   vmm        hipMemCreate / hipMemRelease (virtual memory management handles)
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstring>

namespace {

enum Kind { kMalloc, kManaged, kPitch, k3d, kExt, kAsync, kVmm };

struct Slot {
  void* p = nullptr;
  hipMemGenericAllocationHandle_t h{};
  bool live = false;
};

hipStream_t g_stream = nullptr;
size_t g_gran = 1;

int alloc(Kind k, Slot& s, size_t n) {
  hipError_t e = hipSuccess;
  switch (k) {
    case kMalloc: e = hipMalloc(&s.p, n); break;
    case kManaged: e = hipMallocManaged(&s.p, n, hipMemAttachGlobal); break;
    case kPitch: {
      size_t pitch = 0;
      e = hipMallocPitch(&s.p, &pitch, 1u << 20, n >> 20);
      break;
    }
    case k3d: {
      hipPitchedPtr pp{};
      e = hipMalloc3D(&pp, make_hipExtent(1u << 20, n >> 20, 1));
      s.p = pp.ptr;
      break;
    }
    case kExt: e = hipExtMallocWithFlags(&s.p, n, hipDeviceMallocDefault); break;
    case kAsync:
      e = hipMallocAsync(&s.p, n, g_stream);
      if (e == hipSuccess) e = hipStreamSynchronize(g_stream);
      break;
    case kVmm: {
      hipMemAllocationProp prop{};
      prop.type = hipMemAllocationTypePinned;
      prop.location.type = hipMemLocationTypeDevice;
      prop.location.id = 0;
      e = hipMemCreate(&s.h, (n + g_gran - 1) / g_gran * g_gran, &prop, 0);
      break;
    }
  }
  s.live = e == hipSuccess;
  return (int)e;
}

int release(Kind k, Slot& s) {
  if (!s.live) return 0;
  hipError_t e = hipSuccess;
  switch (k) {
    case kVmm: e = hipMemRelease(s.h); break;
    case kAsync: {
      e = hipFreeAsync(s.p, g_stream);
      if (e == hipSuccess) e = hipStreamSynchronize(g_stream);
      hipMemPool_t pool = nullptr;
      if (e == hipSuccess) e = hipDeviceGetDefaultMemPool(&pool, 0);
      if (e == hipSuccess) e = hipMemPoolTrimTo(pool, 0);
      break;
    }
    default: e = hipFree(s.p); break;
  }
  s.live = false;
  return (int)e;
}

}  // namespace

int main(int argc, char** argv) {
  const char* name = argc > 1 ? argv[1] : "malloc";
  const struct {
    const char* n;
    Kind k;
  } kinds[] = {{"malloc", kMalloc}, {"managed", kManaged}, {"pitch", kPitch}, {"3d", k3d},
               {"ext", kExt},       {"async", kAsync},     {"vmm", kVmm}};
  Kind k = kMalloc;
  bool found = false;
  for (const auto& e : kinds)
    if (!strcmp(name, e.n)) k = e.k, found = true;
  if (!found) {
    fprintf(stderr, "unknown kind %s\n", name);
    return 2;
  }
  if (k == kAsync && hipStreamCreate(&g_stream) != hipSuccess) return 3;
  if (k == kVmm) {
    hipMemAllocationProp prop{};
    prop.type = hipMemAllocationTypePinned;
    prop.location.type = hipMemLocationTypeDevice;
    prop.location.id = 0;
    if (hipMemGetAllocationGranularity(&g_gran, &prop, hipMemAllocationGranularityMinimum) != hipSuccess ||
        g_gran == 0)
      return 4;
  }
  // Sizes relative to what the device (the vGPU quota) has left after setup: a stream's
  // hardware queue carries per-process runtime memory (its context-save area is hundreds
  // of MiB on 256 CUs) that the shim charges to the quota as "context", like the
  // reference charges the primary context. 3/4 fits, +1/2 does not, 1/2 fits after the
  // free. Under a 2 GiB quota with no queue: 1.5 GiB, 1 GiB, 1 GiB.
  size_t free0 = 0, total0 = 0;
  if (hipMemGetInfo(&free0, &total0) != hipSuccess) return 5;
  const size_t unit = 2ull << 20;
  const size_t big = free0 / 4 * 3 / unit * unit, half = free0 / 2 / unit * unit;
  Slot a, b, d;
  int r1 = alloc(k, a, big);
  int r2 = alloc(k, b, half);
  int f1 = release(k, a);
  int r3 = alloc(k, d, half);
  size_t free_b = 0, total_b = 0;
  (void)hipMemGetInfo(&free_b, &total_b);
  printf("{\"kind\": \"%s\", \"r1\": %d, \"r2\": %d, \"f1\": %d, \"r3\": %d, \"free0\": %zu, \"free\": %zu, "
         "\"total\": %zu}\n",
         name, r1, r2, f1, r3, free0, free_b, total_b);
  release(k, b);
  release(k, d);
  if (g_stream) (void)hipStreamDestroy(g_stream);
  return 0;
}
