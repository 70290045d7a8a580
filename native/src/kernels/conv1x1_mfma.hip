// 1x1 convolution on gfx950 matrix cores with the benchmark models' inference epilogues
// fused into the output pass (bf16 NHWC in/out, fp32 accumulate).
//
// A 1x1 convolution over a channels-last activation is a GEMM: X[M = N*H*W, K = Cin]
// times W[Cout, K]^T. In the pre-activation ResNet every such conv is followed by an
// elementwise pass over its output:
//
//   conv1 -> BN + ReLU                          y = act(acc * s[n] + t[n])          (epi 1)
//   conv3 -> + shortcut -> next BN + ReLU       x = acc + r ; y = act(x * s + t)    (epi 2)
//                                               (+ x itself for the next identity
//                                                shortcut)                           (epi 3)
//
// Run separately (library conv + fused_bn_act.hip) the epilogue re-reads the conv output
// from HBM and writes it again; here it is applied while the accumulator tile is still
// on chip, so the conv output never makes the round trip (profiles/r1g: the epilogue
// passes were 33 % of the ResNet-V2-50 inference step).
//
// Kernel shape (CDNA4-first, not a CUDA warp tiling):
//   * 256 threads = 4 wave64s; block tile 128 (M) x BN (64 or 128), K-step 64.
//   * v_mfma_f32_16x16x32_bf16: each wave owns a (128/WM) x (BN/WN) sub-tile as
//     FM x FN 16x16 accumulators. Both operands are K-contiguous, so one lane's
//     fragment (8 consecutive k of one row) is a single 16-byte LDS read.
//   * Global -> registers -> LDS staging, double-buffered: the next K-tile's loads are in
//     flight while the current one feeds the MFMAs; one barrier per K-step.
//   * LDS rows are 128 B (64 bf16); the 16-B chunk index is XOR-swizzled with
//     (row >> 1) & 7 so the 16 lanes of a ds_read_b128 phase hit 16 distinct 16-B slots
//     of the 256-B bank row (conflict-free), for reads and for the staging writes.
//   * Epilogue: the fp32 tile goes through LDS (re-using the staging buffers) so every
//     lane then handles 8 consecutive channels of one pixel: 16-B residual loads and
//     16-B output stores, fully coalesced, per-channel scale/shift in fp32.
//   * XCD-aware tile order: blocks are dispatched round-robin over the 8 XCDs, so the
//     block id is remapped (bijectively) such that the N-tiles of one M-tile run on the
//     same XCD and share its L2 copy of the activation rows.
//
// Requirements (checked on the host): K % 64 == 0, Cout % 64 == 0, 16-byte aligned
// pointers, M*K and M*Cout below 2^34 elements. Rows past M are clamped on load (they
// read a valid row) and never stored.
//
// C ABI (ctypes): pointers are device pointers, `stream` a hipStream_t.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using bf16x8 = __bf16 __attribute__((ext_vector_type(8)));

constexpr int kBM = 128;
constexpr int kBK = 64;
constexpr int kThreads = 256;

__device__ __forceinline__ unsigned swz(unsigned row, unsigned chunk) { return chunk ^ ((row >> 1) & 7u); }

__device__ __forceinline__ float bf_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  __hip_bfloat16 a = __float2bfloat16(lo);
  __hip_bfloat16 b = __float2bfloat16(hi);
  return (unsigned)__bfloat16_as_ushort(a) | ((unsigned)__bfloat16_as_ushort(b) << 16);
}

template <int kAct>
__device__ __forceinline__ float act(float v) {
  if constexpr (kAct == 1) return fmaxf(v, 0.0f);
  if constexpr (kAct == 2) return fminf(fmaxf(v, 0.0f), 6.0f);
  return v;
}

// Bijective block -> tile remap: consecutive tiles (the N-tiles of one M-tile) land on
// the same XCD (hardware dispatches block b to XCD b % 8).
__device__ __forceinline__ unsigned xcd_remap(unsigned bid, unsigned ntiles) {
  const unsigned xcd = bid & 7u, q = ntiles >> 3, r = ntiles & 7u;
  return (xcd < r ? xcd * (q + 1u) : r * (q + 1u) + (xcd - r) * q) + (bid >> 3);
}

// kEpi: 0 plain (y = acc), 1 y = act(acc*s+t), 2 x = acc + r; y = act(x*s+t),
//       3 as 2 and also writes x (bf16) to `sum`.
template <int BN, int WM, int WN, int kEpi, int kAct>
__global__ void __launch_bounds__(kThreads) conv1x1_kernel(const u32x4* __restrict__ A, const u32x4* __restrict__ W,
                                                          const float* __restrict__ scale,
                                                          const float* __restrict__ shift,
                                                          const u32x4* __restrict__ R, u32x4* __restrict__ Y,
                                                          u32x4* __restrict__ S, unsigned M, unsigned N, unsigned K,
                                                          unsigned tiles_n, unsigned ntiles) {
  static_assert(WM * WN == kThreads / 64, "4 waves");
  constexpr int FM = kBM / WM / 16;
  constexpr int FN = BN / WN / 16;
  constexpr int kAStage = kBM * kBK * 2;  // bytes per buffer
  constexpr int kWStage = BN * kBK * 2;
  constexpr int kStage = 2 * (kAStage + kWStage);
  constexpr int kCStride = BN + 4;  // fp32 epilogue tile row stride (16-B multiple)
  constexpr int kEpiBytes = kBM * kCStride * 4;
  constexpr int kLds = kStage > kEpiBytes ? kStage : kEpiBytes;
  constexpr int kALoads = kBM * 8 / kThreads;  // 16-B chunks per thread per K-tile
  constexpr int kWLoads = BN * 8 / kThreads;
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLds];

  const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const unsigned tile = xcd_remap(blockIdx.x, ntiles);
  const unsigned m0 = (tile / tiles_n) * kBM, n0 = (tile % tiles_n) * BN;
  const size_t kvec = K >> 3;  // row stride of A and W in 16-B chunks

  // Buffer b of each operand (computed, not a pointer table: a table of LDS addresses
  // would be a static initializer, which the AMDGPU backend cannot emit).
  auto a_lds = [&](int b) { return reinterpret_cast<u32x4*>(smem + b * kAStage); };
  auto w_lds = [&](int b) { return reinterpret_cast<u32x4*>(smem + 2 * kAStage + b * kWStage); };

  // Per-thread staging sources (row, chunk) are fixed across K-tiles; only the k offset moves.
  const u32x4* a_src[kALoads];
  unsigned a_dst[kALoads];
#pragma unroll
  for (int i = 0; i < kALoads; i++) {
    const unsigned c = tid + i * kThreads, r = c >> 3, ch = c & 7u;
    const unsigned gm = (m0 + r < M) ? m0 + r : M - 1u;
    a_src[i] = A + (size_t)gm * kvec + ch;
    a_dst[i] = r * 8u + swz(r, ch);
  }
  const u32x4* w_src[kWLoads];
  unsigned w_dst[kWLoads];
#pragma unroll
  for (int i = 0; i < kWLoads; i++) {
    const unsigned c = tid + i * kThreads, r = c >> 3, ch = c & 7u;
    w_src[i] = W + (size_t)(n0 + r) * kvec + ch;
    w_dst[i] = r * 8u + swz(r, ch);
  }

  u32x4 ra[kALoads], rw[kWLoads];
  auto load_tile = [&](unsigned kt) {
    const size_t off = (size_t)kt * (kBK / 8);
#pragma unroll
    for (int i = 0; i < kALoads; i++) ra[i] = a_src[i][off];
#pragma unroll
    for (int i = 0; i < kWLoads; i++) rw[i] = w_src[i][off];
  };
  auto store_tile = [&](int b) {
#pragma unroll
    for (int i = 0; i < kALoads; i++) a_lds(b)[a_dst[i]] = ra[i];
#pragma unroll
    for (int i = 0; i < kWLoads; i++) w_lds(b)[w_dst[i]] = rw[i];
  };

  const unsigned wm = wave / WN, wn = wave % WN;
  const unsigned row_base = wm * (kBM / WM), col_base = wn * (BN / WN);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  const unsigned nk = K / kBK;
  load_tile(0);
  store_tile(0);
  __syncthreads();
  for (unsigned kt = 0; kt < nk; kt++) {
    const int cur = kt & 1;
    if (kt + 1 < nk) load_tile(kt + 1);
#pragma unroll
    for (int kk = 0; kk < kBK / 32; kk++) {
      const unsigned chunk = kk * 4u + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
#pragma unroll
      for (int i = 0; i < FM; i++) {
        const unsigned r = row_base + i * 16u + (lane & 15u);
        af[i] = __builtin_bit_cast(bf16x8, a_lds(cur)[r * 8u + swz(r, chunk)]);
      }
#pragma unroll
      for (int j = 0; j < FN; j++) {
        const unsigned r = col_base + j * 16u + (lane & 15u);
        bfr[j] = __builtin_bit_cast(bf16x8, w_lds(cur)[r * 8u + swz(r, chunk)]);
      }
#pragma unroll
      for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
    if (kt + 1 < nk) store_tile(cur ^ 1);
    __syncthreads();
  }

  // Accumulators -> LDS (fp32, row-major [128][BN + 4]); C/D map of 16x16x32:
  // col = lane & 15, row = 4 * (lane >> 4) + reg.
  float* const ctile = reinterpret_cast<float*>(smem);
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int j = 0; j < FN; j++)
#pragma unroll
      for (int r = 0; r < 4; r++)
        ctile[(row_base + i * 16u + 4u * (lane >> 4) + r) * kCStride + col_base + j * 16u + (lane & 15u)] =
            acc[i][j][r];
  __syncthreads();

  const size_t nvec = N >> 3;  // output row stride in 16-B chunks
  constexpr unsigned kChunksPerRow = BN / 8;
#pragma unroll 2
  for (unsigned c = tid; c < kBM * kChunksPerRow; c += kThreads) {
    const unsigned r = c / kChunksPerRow, cc = c % kChunksPerRow;
    const unsigned gm = m0 + r;
    if (gm >= M) continue;
    const float4 v0 = *reinterpret_cast<const float4*>(ctile + r * kCStride + cc * 8u);
    const float4 v1 = *reinterpret_cast<const float4*>(ctile + r * kCStride + cc * 8u + 4u);
    float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const unsigned n = n0 + cc * 8u;
    const size_t o = (size_t)gm * nvec + (n >> 3);
    if constexpr (kEpi >= 2) {
      const u32x4 rv = __builtin_nontemporal_load(&R[o]);
#pragma unroll
      for (int k = 0; k < 4; k++) {
        v[2 * k] += bf_lo(rv[k]);
        v[2 * k + 1] += bf_hi(rv[k]);
      }
      if constexpr (kEpi == 3) {
        u32x4 sv;
#pragma unroll
        for (int k = 0; k < 4; k++) sv[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
        S[o] = sv;
      }
    }
    if constexpr (kEpi >= 1) {
      const float4 s0 = *reinterpret_cast<const float4*>(scale + n);
      const float4 s1 = *reinterpret_cast<const float4*>(scale + n + 4);
      const float4 t0 = *reinterpret_cast<const float4*>(shift + n);
      const float4 t1 = *reinterpret_cast<const float4*>(shift + n + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] = act<kAct>(fmaf(v[k], sc[k], sh[k]));
    }
    u32x4 yv;
#pragma unroll
    for (int k = 0; k < 4; k++) yv[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
    Y[o] = yv;
  }
}

template <int BN, int WM, int WN, int kEpi, int kAct>
int launch(const void* a, const void* w, const float* scale, const float* shift, const void* r, void* y, void* s,
           unsigned M, unsigned N, unsigned K, hipStream_t stream) {
  const unsigned tiles_m = (M + kBM - 1) / kBM, tiles_n = N / BN, ntiles = tiles_m * tiles_n;
  hipLaunchKernelGGL((conv1x1_kernel<BN, WM, WN, kEpi, kAct>), dim3(ntiles), dim3(kThreads), 0, stream,
                     static_cast<const u32x4*>(a), static_cast<const u32x4*>(w), scale, shift,
                     static_cast<const u32x4*>(r), static_cast<u32x4*>(y), static_cast<u32x4*>(s), M, N, K, tiles_n,
                     ntiles);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int BN, int WM, int WN, int kAct>
int by_epi(int epi, const void* a, const void* w, const float* scale, const float* shift, const void* r, void* y,
           void* s, unsigned M, unsigned N, unsigned K, hipStream_t st) {
  switch (epi) {
    case 0: return launch<BN, WM, WN, 0, 0>(a, w, scale, shift, r, y, s, M, N, K, st);
    case 1: return launch<BN, WM, WN, 1, kAct>(a, w, scale, shift, r, y, s, M, N, K, st);
    case 2: return launch<BN, WM, WN, 2, kAct>(a, w, scale, shift, r, y, s, M, N, K, st);
    case 3: return launch<BN, WM, WN, 3, kAct>(a, w, scale, shift, r, y, s, M, N, K, st);
    default: return -1;
  }
}

template <int BN, int WM, int WN>
int by_act(int act, int epi, const void* a, const void* w, const float* scale, const float* shift, const void* r,
           void* y, void* s, unsigned M, unsigned N, unsigned K, hipStream_t st) {
  switch (act) {
    case 0: return by_epi<BN, WM, WN, 0>(epi, a, w, scale, shift, r, y, s, M, N, K, st);
    case 1: return by_epi<BN, WM, WN, 1>(epi, a, w, scale, shift, r, y, s, M, N, K, st);
    case 2: return by_epi<BN, WM, WN, 2>(epi, a, w, scale, shift, r, y, s, M, N, K, st);
    default: return -1;
  }
}

}  // namespace

extern "C" {

// y[M, N] = epilogue(x[M, K] . w[N, K]^T), bf16 row-major (NHWC activations, [Cout, Cin]
// weights), fp32 accumulation. epi: 0 plain, 1 act(acc*scale+shift), 2 act((acc+r)*scale
// + shift), 3 as 2 and sum = acc + r. act: 0 none, 1 relu, 2 relu6. scale/shift: fp32[N].
// Returns 0 on success, -1 on bad arguments, -2 on launch failure.
int vgpu_conv1x1_bf16(const void* x, const void* w, const float* scale, const float* shift, const void* r, void* y,
                      void* sum, int64_t M, int N, int K, int epi, int act, void* stream) {
  if (!x || !w || !y || M <= 0 || N <= 0 || K <= 0 || N % 64 || K % kBK) return -1;
  if (epi < 0 || epi > 3 || act < 0 || act > 2) return -1;
  if (epi >= 1 && (!scale || !shift)) return -1;
  if (epi >= 2 && !r) return -1;
  if (epi == 3 && !sum) return -1;
  if (M >= ((int64_t)1 << 32) || M * (int64_t)K >= ((int64_t)1 << 34) || M * (int64_t)N >= ((int64_t)1 << 34))
    return -1;
  auto misaligned = [](const void* p) { return p && (reinterpret_cast<uintptr_t>(p) & 15u); };
  if (misaligned(x) || misaligned(w) || misaligned(y) || misaligned(r) || misaligned(sum) || misaligned(scale) ||
      misaligned(shift))
    return -1;
  hipStream_t st = static_cast<hipStream_t>(stream);
  const unsigned m = (unsigned)M, n = (unsigned)N, k = (unsigned)K;
  if (N % 128 == 0) return by_act<128, 2, 2>(act, epi, x, w, scale, shift, r, y, sum, m, n, k, st);
  return by_act<64, 4, 1>(act, epi, x, w, scale, shift, r, y, sum, m, n, k, st);
}

}  // extern "C"
