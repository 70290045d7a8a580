// ResNet stem on gfx950 matrix cores, fused end to end:
//
//   pre = relu(bn(maxpool3x3/2(conv7x7/2(x))))      x: [N, H, W, 3] bf16 NHWC, 64 outputs
//
// Run as library kernels the stem is the worst-shaped part of the network: a 3-channel
// convolution (no library tiling fits K = 147) writes a 173x173x64 map per image
// (191 MB at batch 50) that max-pool reads back and shrinks 4x, and the first block's
// BN + ReLU reads the pooled map once more (profiles/r1p: conv 170 us + pool 118 us +
// BN 8 us per ResNet-V2-50 step). Here one block computes an 8x8 tile of pooled outputs:
//
//   1. its 39x39x3 input window is staged in LDS as planar [c][row][col] (zero padding
//      at the image border; one thread per input pixel), the 64x192 weight matrix next
//      to it;
//   2. the 17x17 conv outputs under the tile (pool windows overlap by one conv row, so
//      1.13x recompute) are a [289, K] x [K, 64] GEMM on v_mfma_f32_16x16x32_bf16 with
//      K ordered (kh, c, kw) and kw padded 7 -> 8: a lane's 8-element fragment is then 8
//      consecutive input columns of one (kh, c) row, i.e. four aligned 4-byte LDS reads
//      (the stride-2 conv makes every fragment start on an even column);
//      K = 7 x 3 groups of 8 (+3 zero groups) = 192 = 6 MFMA k-steps;
//      the product is computed transposed (weights as the A operand) so each lane holds
//      4 consecutive channels of one pixel;
//   3. the conv tile is rounded to bf16 into LDS (as the library conv would store it),
//      max-pooled over 3x3/2 with -inf padding, and BN + ReLU applied in fp32; each lane
//      writes 8 channels of one pooled pixel with a 16-byte store.
//
// Only the pooled activation (48 MB at batch 50) ever reaches HBM. Shapes are fixed to the
// ResNet stem (7x7/2 pad 3, 3 -> 64 channels, pool 3x3/2 pad 1); the host checks them.
//
// C ABI (ctypes): pointers are device pointers, `stream` a hipStream_t.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using bf16x8 = __bf16 __attribute__((ext_vector_type(8)));

constexpr int kCin = 3, kCout = 64, kKs = 7;
constexpr int kGroups = 24;                   // K groups of 8 (kh, c) pairs: 21 real + 3 zero
constexpr int kRealGroups = kKs * kCin;       // 21
constexpr int kPT = 8;                        // pooled tile edge
constexpr int kCT = 2 * kPT + 1;              // conv tile edge (17)
constexpr int kIT = 2 * kCT + 5;              // input tile edge (39)
constexpr int kIP = 40;                       // input tile pitch (elements); column 39 is read by the kw=7 pad tap
constexpr int kCPix = kCT * kCT;              // 289 conv pixels
constexpr int kMFrags = (kCPix + 15) / 16;    // 19
constexpr int kCTP = 72;                      // conv tile pitch per pixel (bf16 elements; 144 B)
constexpr int kPatchBytes = kCin * kIT * kIP * 2;           // 9360
constexpr int kWBytes = kCout * kGroups * 16;               // 24576
constexpr int kCTileBytes = kCPix * kCTP * 2;               // 41616
constexpr int kLds = (kPatchBytes + kWBytes) > kCTileBytes ? (kPatchBytes + kWBytes) : kCTileBytes;
constexpr int kThreads = 256;

__device__ __forceinline__ float bf_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

// Two floats -> packed bf16 pair (round to nearest even) in one v_cvt_pk_bf16_f32.
__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  using f32x2_t = float __attribute__((ext_vector_type(2)));
  using bf16x2_t = __bf16 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

__device__ __forceinline__ void stem_tile(const unsigned short* __restrict__ X, const u32x4* __restrict__ Wk,
                                          const float* __restrict__ scale, const float* __restrict__ shift,
                                          u32x4* __restrict__ Y, unsigned H, unsigned W, unsigned CH, unsigned CW,
                                          unsigned PH, unsigned PW, unsigned tiles_x, unsigned tiles_per_img,
                                          unsigned bid) {
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLds];
  unsigned short* const patch = reinterpret_cast<unsigned short*>(smem);       // [3][39][40]
  u32x4* const wl = reinterpret_cast<u32x4*>(smem + kPatchBytes);              // [64][24] 16-B groups
  unsigned short* const ctile = reinterpret_cast<unsigned short*>(smem);       // [289][72] after the GEMM

  const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const unsigned img = bid / tiles_per_img, t = bid - img * tiles_per_img;
  const unsigned ty = t / tiles_x, tx = t - ty * tiles_x;
  const int py0 = (int)(ty * kPT), px0 = (int)(tx * kPT);
  const int ir0 = 4 * py0 - 5, ic0 = 4 * px0 - 5;  // input window origin (conv row 2*py0-1)

  // 1. Input window: each thread stages whole input pixels (3 consecutive bf16, one
  //    address computation per pixel), stored planar; padding and out-of-image pixels are
  //    zero. All of a thread's loads are issued before any is used (an out-of-window pixel
  //    loads a valid address and is zeroed afterwards, so no branch separates the loads):
  //    a load -> store loop would pay one memory latency per element.
  const unsigned short* const ximg = X + (size_t)img * H * W * kCin;
  constexpr unsigned kPix = kIT * kIP, kPer = (kPix + kThreads - 1) / kThreads;
  unsigned short pv[kPer][kCin];
  unsigned pdst[kPer];
#pragma unroll
  for (unsigned q = 0; q < kPer; q++) {
    const unsigned e0 = tid + q * kThreads, e = e0 < kPix ? e0 : kPix - 1u;
    const unsigned r = e / kIP, col = e - r * kIP;
    const int ih = ir0 + (int)r, iw = ic0 + (int)col;
    const bool ok = (unsigned)ih < H && (unsigned)iw < W;
    const unsigned short* src = ximg + (ok ? ((size_t)ih * W + (unsigned)iw) * kCin : 0);
#pragma unroll
    for (int c = 0; c < kCin; c++) {
      const unsigned short v = src[c];
      pv[q][c] = ok ? v : (unsigned short)0;
    }
    pdst[q] = e0 < kPix ? r * kIP + col : ~0u;
  }
  constexpr unsigned kWPer = kCout * kGroups / kThreads;
  static_assert(kWPer * kThreads == kCout * kGroups, "whole weight loads");
  u32x4 wv[kWPer];
#pragma unroll
  for (unsigned q = 0; q < kWPer; q++) wv[q] = Wk[tid + q * kThreads];
#pragma unroll
  for (unsigned q = 0; q < kPer; q++)
    if (pdst[q] != ~0u) {
#pragma unroll
      for (int c = 0; c < kCin; c++) patch[c * (kIT * kIP) + pdst[q]] = pv[q][c];
    }
#pragma unroll
  for (unsigned q = 0; q < kWPer; q++) wl[tid + q * kThreads] = wv[q];
  __syncthreads();

  // 2. Conv tile GEMM, computed transposed (D = W . patch^T): lane l16 is a conv pixel
  //    and the accumulator registers run over channels, so each lane ends up holding 4
  //    consecutive channels of one pixel (one packed 8-byte LDS store per fragment in
  //    step 3a instead of four 2-byte ones). The operand reads are the same as for the
  //    untransposed product: the weight fragment (row = channel) is the A operand, the
  //    patch fragment (column = pixel) the B operand. Wave w owns pixel fragments w, w+4,
  //    ... (wave-uniform guard).
  const unsigned h = lane >> 4, l16 = lane & 15u;
  f32x4 acc[5][4];
#pragma unroll
  for (int i = 0; i < 5; i++)
#pragma unroll
    for (int j = 0; j < 4; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  unsigned pix_off[5];  // this lane's pixel of fragment i, as an offset into a patch row
#pragma unroll
  for (int i = 0; i < 5; i++) {
    unsigned p = (wave + 4u * i) * 16u + l16;
    p = p < (unsigned)kCPix ? p : (unsigned)kCPix - 1u;
    const unsigned crl = p / kCT, ccl = p - crl * kCT;
    pix_off[i] = 2u * crl * kIP + 2u * ccl;
  }
#pragma unroll
  for (int kk = 0; kk < kGroups / 4; kk++) {
    const unsigned g = kk * 4u + h;            // this lane's K group
    const bool real = g < (unsigned)kRealGroups;
    const unsigned gg = real ? g : 0u;         // zero groups read a valid address, then zeroed
    const unsigned kh = gg / kCin, c = gg - kh * kCin;
    const unsigned short* const prow = patch + (c * kIT + kh) * kIP;
    bf16x8 wfr[4];
#pragma unroll
    for (int j = 0; j < 4; j++) wfr[j] = __builtin_bit_cast(bf16x8, wl[(j * 16u + l16) * kGroups + g]);
#pragma unroll
    for (int i = 0; i < 5; i++) {
      const unsigned mf = wave + 4u * i;
      if (mf >= (unsigned)kMFrags) continue;
      const unsigned* src = reinterpret_cast<const unsigned*>(prow + pix_off[i]);
      u32x4 a{src[0], src[1], src[2], src[3]};
      if (!real) a = u32x4{0u, 0u, 0u, 0u};
      const bf16x8 pf = __builtin_bit_cast(bf16x8, a);
#pragma unroll
      for (int j = 0; j < 4; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wfr[j], pf, acc[i][j], 0, 0, 0);
    }
  }
  __syncthreads();  // the conv tile aliases the input window and weights

  // 3a. Conv tile -> LDS as bf16. Transposed C/D map: pixel = l16 of fragment i,
  //     channels 16 j + 4 h + r (r = 0..3) in the lane's 4 registers.
#pragma unroll
  for (int i = 0; i < 5; i++) {
    const unsigned mf = wave + 4u * i;
    if (mf >= (unsigned)kMFrags) continue;
    const unsigned p = mf * 16u + l16;
    if (p >= (unsigned)kCPix) continue;
#pragma unroll
    for (int j = 0; j < 4; j++) {
      uint2 v;
      v.x = pack_bf16(acc[i][j][0], acc[i][j][1]);
      v.y = pack_bf16(acc[i][j][2], acc[i][j][3]);
      *reinterpret_cast<uint2*>(ctile + p * kCTP + j * 16u + 4u * h) = v;
    }
  }
  __syncthreads();

  // 3b. Max-pool 3x3/2 (pad 1, -inf) + BN + ReLU: 64 pooled pixels x 8 channel chunks.
  for (unsigned item = tid; item < (unsigned)(kPT * kPT * (kCout / 8)); item += kThreads) {
    const unsigned pp = item >> 3, ch8 = item & 7u, pyl = pp / kPT, pxl = pp - pyl * kPT;
    const unsigned py = (unsigned)py0 + pyl, px = (unsigned)px0 + pxl;
    if (py >= PH || px >= PW) continue;
    float m[8];
#pragma unroll
    for (int k = 0; k < 8; k++) m[k] = -__builtin_inff();
#pragma unroll
    for (int dy = 0; dy < 3; dy++) {
      const unsigned crl = 2u * pyl + dy;
      const int cr = 2 * py0 - 1 + (int)crl;
      if ((unsigned)cr >= CH) continue;
#pragma unroll
      for (int dx = 0; dx < 3; dx++) {
        const unsigned ccl = 2u * pxl + dx;
        const int cc = 2 * px0 - 1 + (int)ccl;
        if ((unsigned)cc >= CW) continue;
        const u32x4 v = *reinterpret_cast<const u32x4*>(ctile + (crl * kCT + ccl) * kCTP + ch8 * 8u);
#pragma unroll
        for (int k = 0; k < 4; k++) {
          m[2 * k] = fmaxf(m[2 * k], bf_lo(v[k]));
          m[2 * k + 1] = fmaxf(m[2 * k + 1], bf_hi(v[k]));
        }
      }
    }
    const float4 s0 = *reinterpret_cast<const float4*>(scale + ch8 * 8u);
    const float4 s1 = *reinterpret_cast<const float4*>(scale + ch8 * 8u + 4u);
    const float4 t0 = *reinterpret_cast<const float4*>(shift + ch8 * 8u);
    const float4 t1 = *reinterpret_cast<const float4*>(shift + ch8 * 8u + 4u);
    const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
    const float sh[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
    u32x4 yv;
#pragma unroll
    for (int k = 0; k < 4; k++)
      yv[k] = pack_bf16(fmaxf(fmaf(m[2 * k], sc[2 * k], sh[2 * k]), 0.f),
                        fmaxf(fmaf(m[2 * k + 1], sc[2 * k + 1], sh[2 * k + 1]), 0.f));
    Y[(((size_t)img * PH + py) * PW + px) * (kCout / 8) + ch8] = yv;
  }
}

// One pooled tile per block (3 blocks per CU: 122 VGPRs, no spill).
__global__ void __launch_bounds__(kThreads, 3) stem_kernel(const unsigned short* __restrict__ X,
                                                          const u32x4* __restrict__ Wk, const float* __restrict__ scale,
                                                          const float* __restrict__ shift, u32x4* __restrict__ Y,
                                                          unsigned H, unsigned W, unsigned CH, unsigned CW,
                                                          unsigned PH, unsigned PW, unsigned tiles_x,
                                                          unsigned tiles_per_img, unsigned ntiles) {
  stem_tile(X, Wk, scale, shift, Y, H, W, CH, CW, PH, PW, tiles_x, tiles_per_img, blockIdx.x);
}

// Persistent variant for a capped grid (CU-masked vGPU: one dispatch round on the slice,
// profiles/r1z). The tile loop raises register use, so it gets its own build (2 blocks
// per CU) instead of slowing down the uncapped kernel.
__global__ void __launch_bounds__(kThreads) stem_kernel_persistent(
    const unsigned short* __restrict__ X, const u32x4* __restrict__ Wk, const float* __restrict__ scale,
    const float* __restrict__ shift, u32x4* __restrict__ Y, unsigned H, unsigned W, unsigned CH, unsigned CW,
    unsigned PH, unsigned PW, unsigned tiles_x, unsigned tiles_per_img, unsigned ntiles) {
  for (unsigned b = blockIdx.x; b < ntiles; b += gridDim.x) {
    stem_tile(X, Wk, scale, shift, Y, H, W, CH, CW, PH, PW, tiles_x, tiles_per_img, b);
    __syncthreads();  // the next tile's input window overwrites this tile's conv image
  }
}

int g_stem_block_cap = 0;  // vgpu_stem_set_block_cap

}  // namespace

extern "C" {

// y[N, PH, PW, 64] = relu(x_pool * scale + shift), x_pool = maxpool3x3/2/pad1(conv7x7/2/pad3(x, w))
// with x [N, H, W, 3] bf16 NHWC and w the [64, 192] bf16 matrix of the conv weight in
// (kh, c, kw8) order (kw padded 7 -> 8, groups 21..23 zero). scale/shift: fp32[64].
// Returns 0 on success, -1 on bad arguments, -2 on launch failure.
int vgpu_stem_bf16(const void* x, const void* w, const float* scale, const float* shift, void* y, int n, int h,
                   int wd, void* stream) {
  if (!x || !w || !scale || !shift || !y || n <= 0 || h < kKs || wd < kKs) return -1;
  if ((int64_t)n * h * wd * kCin >= ((int64_t)1 << 34)) return -1;
  auto misaligned = [](const void* q) { return reinterpret_cast<uintptr_t>(q) & 15u; };
  if (misaligned(w) || misaligned(y) || misaligned(scale) || misaligned(shift) || (reinterpret_cast<uintptr_t>(x) & 1u))
    return -1;
  const unsigned ch = (unsigned)(h + 2 * 3 - kKs) / 2 + 1, cw = (unsigned)(wd + 2 * 3 - kKs) / 2 + 1;
  const unsigned ph = (ch + 2 - 3) / 2 + 1, pw = (cw + 2 - 3) / 2 + 1;
  const unsigned tiles_x = (pw + kPT - 1) / kPT, tiles_y = (ph + kPT - 1) / kPT;
  const uint64_t blocks = (uint64_t)n * tiles_x * tiles_y;
  if (blocks >= (1ull << 31)) return -1;
  unsigned grid = (unsigned)blocks;
  const bool capped = g_stem_block_cap > 0 && (unsigned)g_stem_block_cap < grid;
  if (capped) grid = (unsigned)g_stem_block_cap;
  hipLaunchKernelGGL(capped ? stem_kernel_persistent : stem_kernel, dim3(grid), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const unsigned short*>(x), static_cast<const u32x4*>(w), scale, shift,
                     static_cast<u32x4*>(y), (unsigned)h, (unsigned)wd, ch, cw, ph, pw, tiles_x, tiles_x * tiles_y,
                     (unsigned)blocks);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Caps the stem grid at `blocks` (persistent blocks; 0 = one block per pooled tile).
void vgpu_stem_set_block_cap(int blocks) { g_stem_block_cap = blocks < 0 ? 0 : blocks; }

}  // extern "C"
