// Per-call cost of the HIP entry points the shim gates, from C++ (no interpreter noise):
// linked against libamdhip64 the normal way, so every call goes through the preloaded
// shim's trampolines exactly as a HIP application's would.
//
//   hip_launch_probe [launches] [calls]   -> one JSON line:
//     launch_us      host time per hipLaunchKernel of an empty kernel, launched in batches
//                    of 256 on one stream with a synchronize per batch (what a launch-bound
//                    tenant pays per kernel)
//     gate_ns        time per hipPointerGetAttributes on a device pointer: a host-only
//                    entry point behind the same trampoline and suspend gate, so the
//                    difference to native is the gate's own cost
//     memset_us      time per 4-byte hipMemsetAsync (a "set" gate), batches of 256
// Each figure is the best of 5 rounds.
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdio>
#include <cstdlib>

__global__ void empty_kernel() {}

namespace {

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

#define CHECK(x)                                                          \
  do {                                                                    \
    hipError_t e_ = (x);                                                  \
    if (e_ != hipSuccess) {                                               \
      fprintf(stderr, "%s failed: %s\n", #x, hipGetErrorString(e_));     \
      return 1;                                                           \
    }                                                                     \
  } while (0)

}  // namespace

int main(int argc, char** argv) {
  const int launches = argc > 1 ? atoi(argv[1]) : 100000;
  const int calls = argc > 2 ? atoi(argv[2]) : 1000000;
  constexpr int kBatch = 256;
  hipStream_t s;
  CHECK(hipStreamCreate(&s));
  void* d = nullptr;
  CHECK(hipMalloc(&d, 1 << 20));
  for (int i = 0; i < 2048; i++) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
  CHECK(hipStreamSynchronize(s));

  double best_launch = 1e30, best_gate = 1e30, best_memset = 1e30;
  for (int round = 0; round < 5; round++) {
    double t0 = now_s();
    for (int i = 0; i < launches; i += kBatch) {
      for (int j = 0; j < kBatch; j++) hipLaunchKernelGGL(empty_kernel, dim3(1), dim3(64), 0, s);
      CHECK(hipStreamSynchronize(s));
    }
    double t = (now_s() - t0) / launches * 1e6;
    if (t < best_launch) best_launch = t;

    hipPointerAttribute_t attr;
    t0 = now_s();
    for (int i = 0; i < calls; i++) CHECK(hipPointerGetAttributes(&attr, d));
    t = (now_s() - t0) / calls * 1e9;
    if (t < best_gate) best_gate = t;

    t0 = now_s();
    for (int i = 0; i < launches / 4; i += kBatch) {
      for (int j = 0; j < kBatch; j++) CHECK(hipMemsetAsync(d, 0, 4, s));
      CHECK(hipStreamSynchronize(s));
    }
    t = (now_s() - t0) / (launches / 4) * 1e6;
    if (t < best_memset) best_memset = t;
  }
  printf("{\"launch_us\": %.4f, \"gate_ns\": %.2f, \"memset_us\": %.4f}\n", best_launch, best_gate, best_memset);
  CHECK(hipFree(d));
  CHECK(hipStreamDestroy(s));
  return 0;
}
