// Calibration: for each CU-mask bit i, launch on a stream restricted to bit i
// and record where the workgroups actually ran (XCC_ID, SE, SH, CU from HW_ID).
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>
#include <cstdio>
#include <vector>
#include <set>

__global__ void where(unsigned* out) {
  if (threadIdx.x == 0) {
    unsigned hw = __builtin_amdgcn_s_getreg((4) | (0 << 6) | (31 << 11));   // HW_REG_HW_ID, 32 bits
    unsigned xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | (15 << 11));  // HW_REG_XCC_ID
    out[blockIdx.x * 2] = hw;
    out[blockIdx.x * 2 + 1] = xcc;
  }
}

int main(int argc, char** argv) {
  int nblk = 64;
  unsigned* d; hipMalloc(&d, nblk * 2 * sizeof(unsigned));
  std::vector<unsigned> h(nblk * 2);
  int ncu = 0; hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  printf("cu_count=%d\n", ncu);
  // unmasked: how many distinct (xcc,se,cu)?
  std::set<unsigned> all;
  for (int r = 0; r < 8; r++) {
    hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, 0, d);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    for (int b = 0; b < nblk; b++) all.insert((h[2*b+1] & 0xf) << 16 | ((h[2*b] >> 8) & 0xff));
  }
  printf("unmasked distinct locations over 8x64 blocks: %zu\n", all.size());
  int nbits = argc > 1 ? atoi(argv[1]) : ncu;
  for (int i = 0; i < nbits; i++) {
    std::vector<uint32_t> mask((ncu + 31) / 32, 0);
    mask[i / 32] |= 1u << (i % 32);
    hipStream_t s;
    if (hipExtStreamCreateWithCUMask(&s, mask.size(), mask.data()) != hipSuccess) { printf("bit %d: stream create failed\n", i); continue; }
    hipLaunchKernelGGL(where, dim3(nblk), dim3(64), 0, s, d);
    hipStreamSynchronize(s);
    hipMemcpy(h.data(), d, h.size() * 4, hipMemcpyDeviceToHost);
    std::set<unsigned> locs;
    for (int b = 0; b < nblk; b++) {
      unsigned hw = h[2*b], xcc = h[2*b+1];
      locs.insert((xcc & 0xf) << 16 | ((hw >> 13) & 7) << 8 | ((hw >> 12) & 1) << 4 | ((hw >> 8) & 0xf));
    }
    printf("bit %3d ->", i);
    for (unsigned l : locs) printf(" xcc%u.se%u.sh%u.cu%u", l >> 16, (l >> 8) & 0xff, (l >> 4) & 0xf, l & 0xf);
    printf("\n");
    hipStreamDestroy(s);
  }
  return 0;
}
