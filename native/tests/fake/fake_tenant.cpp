// A tenant library that links HIP (the fake libamdhip64) - what an application module is
// when it is loaded with RTLD_DEEPBIND: its own dependency scope (HIP, then ROCr) comes ahead
// of the preloaded shim (tests/test_loader_bypass.py).
#define __HIP_PLATFORM_AMD__ 1
#include <hip/hip_runtime_api.h>

extern "C" {

// hipMalloc of `bytes` on device 0: 0 on success, the HIP error otherwise.
int tenant_malloc(unsigned long long bytes) {
  if (hipInit(0) != hipSuccess) return -1;
  void* p = nullptr;
  return (int)hipMalloc(&p, (size_t)bytes);
}

// hipMemGetInfo's total (the quota under the shim).
unsigned long long tenant_total() {
  size_t f = 0, t = 0;
  if (hipInit(0) != hipSuccess || hipMemGetInfo(&f, &t) != hipSuccess) return 0;
  return t;
}

// One launch of a 10-microsecond fake kernel on the null stream, then a synchronize: 0 on
// success. (The fake's "kernel" is a uint32 duration in microseconds.)
int tenant_launch() {
  static uint32_t us = 10;
  if (hipInit(0) != hipSuccess) return -1;
  hipError_t e = hipLaunchKernel(&us, dim3(1), dim3(64), nullptr, 0, nullptr);
  return e != hipSuccess ? (int)e : (int)hipDeviceSynchronize();
}

}  // extern "C"
