// gfx950 calibration kernels for the vGPU data plane (test instruments, SURVEY.md
// §2.8: "a calibration kernel that measures CU-mask / temporal-limit fidelity; a
// bandwidth probe for host-spill throughput").
//
//  * vgpu_cu_census   every workgroup records where it ran (XCC id from
//                     HW_REG_XCC_ID, SE/CU from HW_REG_HW_ID) while spinning long
//                     enough that the dispatcher has to spread the grid over every
//                     CU the queue may use: the number of distinct CUs observed is
//                     the spatial partition actually enforced.
//  * vgpu_spin        fixed-duration workgroups (s_memrealtime, 100 MHz) for
//                     duty-cycle / temporal-limit measurements; vgpu_spin_lds the
//                     same holding dynamic LDS (few workgroups per CU at a time).
//  * vgpu_stream_copy 16-byte-per-lane grid-stride copy; with the source in spilled
//                     host memory it measures the oversubscription path's bandwidth.
//  * vgpu_scratch_hog a kernel with a 16 KiB-per-lane private segment (dynamically
//                     indexed, so it lives in scratch): makes ROCr allocate a large
//                     scratch backing store behind the allocation hooks' back, which the
//                     shim's context accounting has to pick up from KFD.
//
// C ABI, loaded with ctypes; pointers are device pointers (e.g. torch data_ptr()) and
// `stream` is a hipStream_t (torch.cuda.current_stream().cuda_stream).
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

constexpr unsigned kHwRegHwId = 4;
constexpr unsigned kHwRegXccId = 20;

__global__ void __launch_bounds__(64) census_kernel(uint32_t* out, uint64_t spin_ticks) {
  if (threadIdx.x == 0) {
    // s_getreg_b32 immediate: id | offset << 6 | (size - 1) << 11
    uint32_t hw = __builtin_amdgcn_s_getreg(kHwRegHwId | (0u << 6) | (31u << 11));
    uint32_t xcc = __builtin_amdgcn_s_getreg(kHwRegXccId | (0u << 6) | (3u << 11));
    uint32_t cu = (hw >> 8) & 0xf;
    uint32_t sh = (hw >> 12) & 0x1;
    uint32_t se = (hw >> 13) & 0x7;
    out[blockIdx.x] = (xcc & 0xf) << 12 | se << 8 | sh << 4 | cu;
    uint64_t t0 = __builtin_amdgcn_s_memrealtime();
    while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(2);
  }
}

__global__ void __launch_bounds__(64) spin_kernel(uint64_t spin_ticks, uint64_t* done) {
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0 && done) atomicAdd(reinterpret_cast<unsigned long long*>(done), 1ull);
}

// Same spin, but each workgroup also holds `dynamic LDS` bytes, so only a few fit on a CU
// at once: the grid has to be dispatched over many rounds (like a GEMM kernel's), which
// exposes dispatcher-level interference between CU-masked queues.
__global__ void __launch_bounds__(64) spin_lds_kernel(uint64_t spin_ticks) {
  extern __shared__ unsigned char dyn_lds[];
  uint64_t t0 = __builtin_amdgcn_s_memrealtime();
  while (__builtin_amdgcn_s_memrealtime() - t0 < spin_ticks) __builtin_amdgcn_s_sleep(1);
  if (threadIdx.x == 0) dyn_lds[0] = 1;
}

constexpr int kScratchWords = 4096;  // 16 KiB of private memory per lane

__global__ void __launch_bounds__(64) scratch_kernel(uint32_t* out, uint32_t stride) {
  uint32_t buf[kScratchWords];
  const uint32_t lane = threadIdx.x;
  // Data-dependent indices keep the array out of registers (stride comes from the host).
  for (int i = 0; i < kScratchWords; i++) buf[(i * stride + lane) % kScratchWords] = i ^ lane;
  uint32_t acc = 0;
  for (int i = 0; i < kScratchWords; i += 7) acc += buf[(i * stride) % kScratchWords];
  out[blockIdx.x * 64 + lane] = acc;
}

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

__global__ void __launch_bounds__(256) copy_kernel(u32x4* __restrict__ dst, const u32x4* __restrict__ src, size_t n) {
  size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
  size_t stride = (size_t)gridDim.x * blockDim.x;
  for (; i < n; i += stride) dst[i] = __builtin_nontemporal_load(&src[i]);
}

}  // namespace

extern "C" {

// Launches `nblocks` single-wave workgroups that each spin `spin_us` microseconds and
// write their location code to out[block] (device buffer of nblocks uint32).
int vgpu_cu_census(uint32_t* out, int nblocks, int spin_us, void* stream) {
  if (!out || nblocks <= 0) return -1;
  hipLaunchKernelGGL(census_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, out,
                     (uint64_t)spin_us * 100);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

int vgpu_spin(int nblocks, int spin_us, uint64_t* done, void* stream) {
  if (nblocks <= 0) return -1;
  hipLaunchKernelGGL(spin_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, (uint64_t)spin_us * 100, done);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// `nblocks` single-wave workgroups spinning `spin_us` each while holding `lds_bytes` of LDS.
int vgpu_spin_lds(int nblocks, int spin_us, int lds_bytes, void* stream) {
  if (nblocks <= 0 || lds_bytes < 1 || lds_bytes > 160 * 1024) return -1;
  hipLaunchKernelGGL(spin_lds_kernel, dim3(nblocks), dim3(64), (size_t)lds_bytes, (hipStream_t)stream,
                     (uint64_t)spin_us * 100);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// `nblocks` single-wave workgroups, each lane with a 16 KiB private array; out holds
// nblocks * 64 uint32. `stride` must be odd (any odd value gives a permutation).
int vgpu_scratch_hog(uint32_t* out, int nblocks, int stride, void* stream) {
  if (!out || nblocks <= 0 || !(stride & 1)) return -1;
  hipLaunchKernelGGL(scratch_kernel, dim3(nblocks), dim3(64), 0, (hipStream_t)stream, out, (uint32_t)stride);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Copies `bytes` (multiple of 16) from src to dst.
int vgpu_stream_copy(void* dst, const void* src, size_t bytes, void* stream) {
  if (!dst || !src || (bytes & 15)) return -1;
  size_t n = bytes / 16;
  // >> 256 CUs x 8 waves: enough workgroups in flight to saturate HBM / the link.
  int blocks = (int)((n + 255) / 256);
  if (blocks > 256 * 16) blocks = 256 * 16;
  if (blocks < 1) blocks = 1;
  hipLaunchKernelGGL(copy_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, (u32x4*)dst, (const u32x4*)src, n);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
