// NHWC convolution on gfx950 matrix cores with the benchmark models' inference epilogues
// fused into the output pass (bf16 in/out, fp32 accumulate).
//
// Over a channels-last activation a convolution is a GEMM: Y[M = N*OH*OW, Cout] =
// im2col(X)[M, K = KH*KW*Cin] . W[Cout, K]^T, with the weight in its channels-last layout
// [Cout][KH][KW][Cin]. A 1x1/stride-1 conv needs no im2col at all (X itself is the
// [M, Cin] operand); every other shape (3x3, strided 1x1 shortcuts) gathers its A tile
// implicitly: a 64-wide K-tile always lies inside one (kh, kw) tap because Cin % 64 == 0,
// so each staged row is one contiguous 128-B piece of one input pixel, or zeros for the
// padding. In the pre-activation ResNet every conv is followed by an elementwise pass:
//
//   conv1, conv2 -> BN + ReLU                   y = act(acc * s[n] + t[n])          (epi 1)
//   conv3 -> + shortcut -> next BN + ReLU       x = acc + r ; y = act(x * s + t)    (epi 2)
//                                               (+ x itself for the next identity
//                                                shortcut)                           (epi 3)
//   MobileNet projection (+ residual after BN)  y = act(acc * s + t + r)            (epi 4)
//   shortcut conv                               y = acc                             (epi 0)
//   conv3 when the next block's conv1 takes     x = acc + r                         (epi 5)
//   its BN + ReLU as a prologue
//
// Prologue: before an identity-shortcut block, the activation pre = relu(bn1(x)) is only
// read by that block's 1x1 conv1. That conv1 then stages relu(x * s + t) itself while
// loading its A tile, and the previous conv3 writes only x (epi 5): one fewer full-size
// activation written and read per block (e.g. 194 MB at stage 1, batch 50).
//
// Run separately (library conv + fused_bn_act.hip) the epilogue re-reads the conv output
// from HBM and writes it again; here it is applied while the accumulator tile is still
// on chip, so the conv output never makes the round trip (profiles/r1g: the epilogue
// passes were 33 % of the ResNet-V2-50 inference step; profiles/r1n: the 1x1 layers alone
// went 1.15-1.65x faster).
//
// Kernel shape (CDNA4-first, not a CUDA warp tiling):
//   * 256 threads = 4 wave64s; block tile BM (128, or 64 when 128-row tiles would leave
//     the chip under-filled) x BN (64 or 128), K-step 64.
//   * v_mfma_f32_16x16x32_bf16: each wave owns a (128/WM) x (BN/WN) sub-tile as
//     FM x FN 16x16 accumulators. Both operands are K-contiguous, so one lane's
//     fragment (8 consecutive k of one row) is a single 16-byte LDS read.
//   * Global -> registers -> LDS staging, double-buffered: the next K-tile's loads are in
//     flight while the current one feeds the MFMAs; one barrier per K-step. Loads go
//     through raw buffer descriptors: a fixed per-thread voffset plus the K position as
//     the scalar soffset, and padding taps get an out-of-range voffset, for which the
//     hardware returns zeros. A select after the load (the first version) made every
//     K-step wait for its loads before the MFMAs and cost ~90 VALU per K-step in 64-bit
//     address arithmetic; now the main loop is ~MFMA + LDS only.
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
// Requirements (checked on the host): Cin % 64 == 0, Cout % 64 == 0, 16-byte aligned
// pointers, the weight and one image's input and output below 2 GiB (larger batches are
// split into several launches). Rows past M are clamped on load (they read a valid row)
// and never stored.
//
// C ABI (ctypes): pointers are device pointers, `stream` a hipStream_t.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdlib>

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using bf16x8 = __bf16 __attribute__((ext_vector_type(8)));

// Cache policy of the epilogue's residual loads / output stores (A/B builds).
#ifndef VGPU_CONV_RES_NT
#define VGPU_CONV_RES_NT 1
#endif
#ifndef VGPU_CONV_Y_NT
#define VGPU_CONV_Y_NT 0
#endif

constexpr int kBK = 64;
constexpr int kThreads = 256;

// Shape of one launch. The tensors travel as separate __restrict__ kernel arguments:
// pointers inside a by-value struct lose `noalias`, and a build that passed them that
// way ran the stage-1 conv3 (+ residual + sum epilogue) in 175 us instead of 139 us.
struct ConvGeom {
  unsigned M, N, K;                             // GEMM: M = Nb*OH*OW, N = Cout, K = KH*KW*C
  unsigned H, W, C, OH, OW, KW, stride, pad;    // geometry (implicit-GEMM path)
  unsigned tiles_n, ntiles;
  unsigned x_bytes, w_bytes;                    // buffer-descriptor ranges (< 2^31, host-checked)
  // Dual source (kDual): K-tiles past K1 = C read X2 [Nb, H2, W2, C2] at pixel
  // (oh * stride2, ow * stride2), a strided 1x1 conv accumulated into the same tile.
  unsigned C2, H2, W2, stride2, x2_bytes;
};

struct ConvArgs {
  const void* x;
  const void* w;
  const float* scale;
  const float* shift;
  const void* r;
  void* y;
  void* s;
  const float* pscale;  // prologue (1x1 path): A = relu(X * pscale + pshift), or null
  const float* pshift;
  const void* x2;       // second A source (dual path), or null
  int max_blocks;       // grid cap (persistent blocks), 0 = one block per tile
  ConvGeom g;
};

__device__ __forceinline__ unsigned swz(unsigned row, unsigned chunk) { return chunk ^ ((row >> 1) & 7u); }

// Raw buffer descriptor over [p, p + bytes) (bytes < 2^31). The inputs are made provably
// wave-uniform so the loads through it are not wrapped in waterfall loops.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  // (readfirstlane returns int: widen through uint32_t, not by sign extension.)
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}

// A voffset at or past every descriptor's range: the hardware range check returns zeros
// (the implicit GEMM's padding taps, without a select after the load).
constexpr unsigned kOOB = 0x80000000u;

// LDS-DMA: 16 B per lane from the buffer straight into LDS at lds + 16 * lane (`lds` is
// wave-uniform), no VGPR destination and no ds_write.
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, u32x4* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (__attribute__((address_space(3))) void*)lds, 16, (int)voff, (int)soff,
                                           0, 0);
}

__device__ __forceinline__ float bf_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

// Two floats -> packed bf16 pair (round to nearest even) in one v_cvt_pk_bf16_f32.
__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  using f32x2_t = float __attribute__((ext_vector_type(2)));
  using bf16x2_t = __bf16 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
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
//       3 as 2 and also writes x (bf16) to `s`, 4 y = act(acc*s + t + r), 5 y = acc + r,
//       6 as 3 without a residual (s = acc; y = act(acc*s+t)).
// kIm2col: false = 1x1/stride-1 (A is X itself), true = implicit GEMM gather.
// kPro (1x1 path): the A operand is relu(X * pscale[c] + pshift[c]) (the consumer's
//       pre-activation BN + ReLU applied to the A fragments as they leave LDS, rounded to
//       bf16 as a separate pass would store it), so the producer never writes that
//       activation to HBM.
// kDual (1x1 path): A = [X | strided X2] along K, W = [W1 | W2]: the ResNet projection
//       block's conv3 and its shortcut conv as one GEMM, so the shortcut output is never
//       written to HBM and read back as the residual.
template <int BM, int BN, int WM, int WN, int kEpi, int kAct, bool kIm2col, bool kPro, bool kDual>
__device__ __forceinline__ void conv_tile(const u32x4* __restrict__ X, const u32x4* __restrict__ X2,
                                          const u32x4* __restrict__ Wt,
                                          const float* __restrict__ scale, const float* __restrict__ shift,
                                          const u32x4* __restrict__ R, u32x4* __restrict__ Y, u32x4* __restrict__ S,
                                          const float* __restrict__ pscale, const float* __restrict__ pshift,
                                          const ConvGeom& p, const unsigned tile) {
  static_assert(!(kPro && kIm2col), "prologue only on the 1x1 path");
  static_assert(WM * WN == kThreads / 64, "4 waves");
  constexpr int FM = BM / WM / 16;
  constexpr int FN = BN / WN / 16;
  constexpr int kAStage = BM * kBK * 2;  // bytes per buffer
  constexpr int kWStage = BN * kBK * 2;
  constexpr int kStage = 2 * (kAStage + kWStage);
  constexpr int kCStride = BN + 4;  // fp32 epilogue tile row stride (16-B multiple)
  constexpr int kEpiBytes = BM * kCStride * 4;
  constexpr int kLdsMain = kStage > kEpiBytes ? kStage : kEpiBytes;
  constexpr int kParam = kPro ? 512 : 0;  // prologue scale | shift of one K-tile (fp32 x 64 x 2)
  constexpr int kLds = kLdsMain + 2 * kParam;
  constexpr int kALoads = BM * 8 / kThreads;  // 16-B chunks per thread per K-tile
  constexpr int kWLoads = BN * 8 / kThreads;
  __shared__ __attribute__((aligned(16))) unsigned char smem[kLds];

  const unsigned M = p.M, N = p.N, K = p.K;
  const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const unsigned m0 = (tile / p.tiles_n) * BM, n0 = (tile % p.tiles_n) * BN;

  // Buffer b of each operand (computed, not a pointer table: a table of LDS addresses
  // would be a static initializer, which the AMDGPU backend cannot emit).
  auto a_lds = [&](int b) { return reinterpret_cast<u32x4*>(smem + b * kAStage); };
  auto w_lds = [&](int b) { return reinterpret_cast<u32x4*>(smem + 2 * kAStage + b * kWStage); };
  auto p_lds = [&](int b) { return reinterpret_cast<u32x4*>(smem + kLdsMain + b * kParam); };

  // Operands are read through buffer descriptors with 32-bit byte offsets: per thread a
  // fixed voffset, the K position as the scalar soffset, so a K-tile's loads cost no
  // vector address arithmetic (the host keeps every launch's tensors below 2 GiB).
  const __amdgpu_buffer_rsrc_t xr = make_rsrc(X, p.x_bytes), wr = make_rsrc(Wt, p.w_bytes);
  const unsigned krow = K * 2u;  // W row in bytes
  unsigned a_vo[kALoads];        // 1x1: row start; im2col: current tap's pixel, or kOOB
  unsigned a_vo2[kDual ? kALoads : 1];  // dual: the strided source-2 pixel's row start
  const __amdgpu_buffer_rsrc_t xr2 = make_rsrc(kDual ? static_cast<const void*>(X2) : X, kDual ? p.x2_bytes : 0u);
  const unsigned nk1 = p.C / kBK;       // K-tiles from source 1
  int a_pix[kALoads], a_ih0[kALoads], a_iw0[kALoads];
  const unsigned cbytes = p.C * 2u;  // input pixel stride (im2col path)
  // Staging is LDS-DMA. Its image is lane-linear (lane l of piece i fills 16-B slot
  // tid + 256 i of the buffer), so the XOR swizzle moves to the source: slot (row r,
  // chunk ch) is loaded from logical chunk swz(r, ch) (the swizzle is an involution).
  const unsigned wv = __builtin_amdgcn_readfirstlane(wave);
#pragma unroll
  for (int i = 0; i < kALoads; i++) {
    const unsigned c = tid + i * kThreads, r = c >> 3, ch = swz(r, c & 7u);
    const unsigned gm = (m0 + r < M) ? m0 + r : M - 1u;
    if constexpr (kIm2col) {
      const unsigned plane = p.OH * p.OW;
      const unsigned img = gm / plane, rem = gm - img * plane;
      const unsigned oh = rem / p.OW, ow = rem - oh * p.OW;
      a_ih0[i] = (int)(oh * p.stride) - (int)p.pad;
      a_iw0[i] = (int)(ow * p.stride) - (int)p.pad;
      // Byte offset of the (possibly padding) pixel (ih0, iw0): may be negative, every
      // in-bounds tap lands inside the tensor.
      a_pix[i] = (int)(((img * p.H) * p.W) * cbytes) + (a_ih0[i] * (int)p.W + a_iw0[i]) * (int)cbytes + (int)(ch * 16u);
      a_vo[i] = kOOB;
    } else {
      a_vo[i] = gm * cbytes + ch * 16u;
      a_pix[i] = a_ih0[i] = a_iw0[i] = 0;
      if constexpr (kDual) {
        const unsigned plane = p.OH * p.OW;
        const unsigned img = gm / plane, rem = gm - img * plane;
        const unsigned oh = rem / p.OW, ow = rem - oh * p.OW;
        a_vo2[i] = ((img * p.H2 + oh * p.stride2) * p.W2 + ow * p.stride2) * (p.C2 * 2u) + ch * 16u;
      }
    }
  }
  unsigned w_vo[kWLoads];
#pragma unroll
  for (int i = 0; i < kWLoads; i++) {
    const unsigned c = tid + i * kThreads, r = c >> 3, ch = swz(r, c & 7u);
    w_vo[i] = (n0 + r) * krow + ch * 16u;
  }
  // Prologue parameters ride along with each K-tile: lanes 0-15 of wave 0 DMA the tile's
  // 64 scales, then its 64 shifts, into the buffer's parameter slot.
  const __amdgpu_buffer_rsrc_t psr = make_rsrc(kPro ? static_cast<const void*>(pscale) : X, kPro ? K * 4u : 0u);
  const __amdgpu_buffer_rsrc_t ptr_ = make_rsrc(kPro ? static_cast<const void*>(pshift) : X, kPro ? K * 4u : 0u);
  // im2col: the K-tile's (kh, kw) tap and channel block, advanced one K-tile per load
  // (wave-uniform scalars). A tap's bounds checks run once per tap, not per K-tile.
  const unsigned cpt = p.C / kBK;
  unsigned t_c0 = 0, t_kw = 0, t_kh = 0;

  // The wave's LDS-DMA destination for piece i of buffer `base`.
  auto slot = [&](u32x4* base, int i) { return base + wv * 64u + (unsigned)i * kThreads; };
  auto load_tile = [&](unsigned kt, int b) {
    const unsigned koff = kt * (kBK * 2u);  // bytes along K
    if constexpr (kPro) {
      if (wv == 0 && lane < 16u) {
        dma16(psr, p_lds(b), lane * 16u, kt * (kBK * 4u));
        dma16(ptr_, p_lds(b) + 16, lane * 16u, kt * (kBK * 4u));
      }
    }
    if constexpr (kIm2col) {
      if (t_c0 == 0) {  // first K-tile of a new tap
        const int toff = ((int)t_kh * (int)p.W + (int)t_kw) * (int)cbytes;
#pragma unroll
        for (int i = 0; i < kALoads; i++) {
          const bool ok = (unsigned)(a_ih0[i] + (int)t_kh) < p.H && (unsigned)(a_iw0[i] + (int)t_kw) < p.W;
          a_vo[i] = ok ? (unsigned)(a_pix[i] + toff) : kOOB;
        }
      }
      const unsigned soff = t_c0 * (kBK * 2u);
#pragma unroll
      for (int i = 0; i < kALoads; i++) dma16(xr, slot(a_lds(b), i), a_vo[i], soff);
      if (++t_c0 == cpt) {
        t_c0 = 0;
        if (++t_kw == p.KW) t_kw = 0, t_kh++;
      }
    } else if (kDual && kt >= nk1) {
      const unsigned koff2 = (kt - nk1) * (kBK * 2u);
#pragma unroll
      for (int i = 0; i < kALoads; i++) dma16(xr2, slot(a_lds(b), i), a_vo2[i], koff2);
    } else {
#pragma unroll
      for (int i = 0; i < kALoads; i++) dma16(xr, slot(a_lds(b), i), a_vo[i], koff);
    }
#pragma unroll
    for (int i = 0; i < kWLoads; i++) dma16(wr, slot(w_lds(b), i), w_vo[i], koff);
  };

  const unsigned wm = wave / WN, wn = wave % WN;
  const unsigned row_base = wm * (BM / WM), col_base = wn * (BN / WN);
  f32x4 acc[FM][FN];
#pragma unroll
  for (int i = 0; i < FM; i++)
#pragma unroll
    for (int j = 0; j < FN; j++) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  auto compute = [&](int b) {
#pragma unroll
    for (int kk = 0; kk < kBK / 32; kk++) {
      const unsigned chunk = kk * 4u + (lane >> 4);
      bf16x8 af[FM], bfr[FN];
      // Prologue: this lane's fragments hold channels 8 * chunk .. + 7 of the K-tile.
      float ps[kPro ? 8 : 1], pt[kPro ? 8 : 1];
      if constexpr (kPro) {
        const float4* pp = reinterpret_cast<const float4*>(p_lds(b));
        const float4 s0 = pp[2 * chunk], s1 = pp[2 * chunk + 1], t0 = pp[16 + 2 * chunk], t1 = pp[17 + 2 * chunk];
        ps[0] = s0.x; ps[1] = s0.y; ps[2] = s0.z; ps[3] = s0.w; ps[4] = s1.x; ps[5] = s1.y; ps[6] = s1.z; ps[7] = s1.w;
        pt[0] = t0.x; pt[1] = t0.y; pt[2] = t0.z; pt[3] = t0.w; pt[4] = t1.x; pt[5] = t1.y; pt[6] = t1.z; pt[7] = t1.w;
      }
#pragma unroll
      for (int i = 0; i < FM; i++) {
        const unsigned r = row_base + i * 16u + (lane & 15u);
        u32x4 v = a_lds(b)[r * 8u + swz(r, chunk)];
        if constexpr (kPro) {
          // relu(x * scale + shift), rounded to bf16 as a separate pass would store it.
#pragma unroll
          for (int k = 0; k < 4; k++)
            v[k] = pack_bf16(fmaxf(fmaf(bf_lo(v[k]), ps[2 * k], pt[2 * k]), 0.f),
                             fmaxf(fmaf(bf_hi(v[k]), ps[2 * k + 1], pt[2 * k + 1]), 0.f));
        }
        af[i] = __builtin_bit_cast(bf16x8, v);
      }
#pragma unroll
      for (int j = 0; j < FN; j++) {
        const unsigned r = col_base + j * 16u + (lane & 15u);
        bfr[j] = __builtin_bit_cast(bf16x8, w_lds(b)[r * 8u + swz(r, chunk)]);
      }
#pragma unroll
      for (int i = 0; i < FM; i++)
#pragma unroll
        for (int j = 0; j < FN; j++) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
    }
  };

  const unsigned nk = K / kBK;
  // The residual tile does not depend on the GEMM: its loads go out with the first
  // K-tile's, so they are in flight together and complete under the MFMAs instead of
  // stalling the epilogue.
  constexpr unsigned kChunksPerRow = BN / 8;
  constexpr int kEpiIters = BM * kChunksPerRow / kThreads;
  static_assert(kEpiIters * kThreads == BM * kChunksPerRow, "whole epilogue iterations");
  const size_t nvec = N >> 3;  // output row stride in 16-B chunks
  constexpr bool kRes = kEpi >= 2 && kEpi <= 5;  // epilogue reads the residual
  u32x4 rpre[kRes ? kEpiIters : 1];
  auto prefetch_residual = [&]() {
    if constexpr (kRes) {
#pragma unroll
      for (int j = 0; j < kEpiIters; j++) {
        const unsigned c = tid + j * kThreads, r = c / kChunksPerRow, cc = c % kChunksPerRow;
        const unsigned gm = (m0 + r < M) ? m0 + r : M - 1u;
#if VGPU_CONV_RES_NT
        rpre[j] = __builtin_nontemporal_load(&R[(size_t)gm * nvec + (n0 >> 3) + cc]);
#else
        rpre[j] = R[(size_t)gm * nvec + (n0 >> 3) + cc];
#endif
      }
    }
  };
  // Step kt: barrier (its vmcnt(0) retires tile kt's LDS-DMA), start tile kt + 1's LDS-DMA
  // into the buffer step kt - 1 read, compute tile kt. A 3-deep ring (two tiles in
  // flight, counted vmcnt + bare s_barrier) was slower on 19 of 23 ResNet-50 layers: it
  // costs a block per CU of LDS (profiles/r1al). So was a transposed product with the
  // epilogue on the accumulators (4 channels of a pixel per lane, no LDS round trip): its
  // 8-byte residual loads and output stores made the memory-bound layers up to 1.6x
  // slower (profiles/r1am).
  prefetch_residual();
  load_tile(0, 0);
  for (unsigned kt = 0; kt < nk; kt++) {
    __syncthreads();
    if (kt + 1 < nk) load_tile(kt + 1, (kt & 1) ^ 1);
    compute(kt & 1);
  }
  __syncthreads();  // every wave's last fragment reads before the epilogue reuses LDS

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

#pragma unroll
  for (int j = 0; j < kEpiIters; j++) {
    const unsigned c = tid + j * kThreads, r = c / kChunksPerRow, cc = c % kChunksPerRow;
    const unsigned gm = m0 + r;
    if (gm >= M) continue;
    const float4 v0 = *reinterpret_cast<const float4*>(ctile + r * kCStride + cc * 8u);
    const float4 v1 = *reinterpret_cast<const float4*>(ctile + r * kCStride + cc * 8u + 4u);
    float v[8] = {v0.x, v0.y, v0.z, v0.w, v1.x, v1.y, v1.z, v1.w};
    const unsigned n = n0 + cc * 8u;
    const size_t o = (size_t)gm * nvec + (n >> 3);
    float rr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
    if constexpr (kRes) {
      const u32x4 rv = rpre[j];
#pragma unroll
      for (int k = 0; k < 4; k++) {
        rr[2 * k] = bf_lo(rv[k]);
        rr[2 * k + 1] = bf_hi(rv[k]);
      }
    }
    if constexpr (kEpi == 2 || kEpi == 3 || kEpi == 5 || kEpi == 6) {
#pragma unroll
      for (int k = 0; k < 8; k++) v[k] += rr[k];
      if constexpr (kEpi == 3 || kEpi == 6) {
        u32x4 sv;
#pragma unroll
        for (int k = 0; k < 4; k++) sv[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
#if VGPU_CONV_Y_NT
        __builtin_nontemporal_store(sv, &S[o]);
#else
        S[o] = sv;
#endif
      }
    }
    if constexpr ((kEpi >= 1 && kEpi <= 4) || kEpi == 6) {
      const float4 s0 = *reinterpret_cast<const float4*>(scale + n);
      const float4 s1 = *reinterpret_cast<const float4*>(scale + n + 4);
      const float4 t0 = *reinterpret_cast<const float4*>(shift + n);
      const float4 t1 = *reinterpret_cast<const float4*>(shift + n + 4);
      const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
      const float sh[8] = {t0.x, t0.y, t0.z, t0.w, t1.x, t1.y, t1.z, t1.w};
#pragma unroll
      for (int k = 0; k < 8; k++) {
        float o_ = fmaf(v[k], sc[k], sh[k]);
        if constexpr (kEpi == 4) o_ += rr[k];
        v[k] = act<kAct>(o_);
      }
    }
    u32x4 yv;
#pragma unroll
    for (int k = 0; k < 4; k++) yv[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
#if VGPU_CONV_Y_NT
    __builtin_nontemporal_store(yv, &Y[o]);
#else
    Y[o] = yv;
#endif
  }
}

// One tile per block, or persistent when the grid is capped below the tile count: on a
// CU-masked vGPU the cap is the slice's block capacity, so the whole grid is placed in
// one round and this tenant's dispatch never waits for room on its slice while holding
// up the other tenants' dispatches (profiles/r1z). The grid is a multiple of 8 when
// capped, so every tile a block visits keeps the block's XCD in xcd_remap.
template <int BM, int BN, int WM, int WN, int kEpi, int kAct, bool kIm2col, bool kPro, bool kDual>
__global__ void __launch_bounds__(kThreads) conv_kernel(const u32x4* __restrict__ X, const u32x4* __restrict__ X2,
                                                       const u32x4* __restrict__ Wt,
                                                       const float* __restrict__ scale, const float* __restrict__ shift,
                                                       const u32x4* __restrict__ R, u32x4* __restrict__ Y,
                                                       u32x4* __restrict__ S, const float* __restrict__ pscale,
                                                       const float* __restrict__ pshift, const ConvGeom p) {
  for (unsigned t = blockIdx.x; t < p.ntiles; t += gridDim.x) {
    conv_tile<BM, BN, WM, WN, kEpi, kAct, kIm2col, kPro, kDual>(X, X2, Wt, scale, shift, R, Y, S, pscale, pshift, p,
                                                      xcd_remap(t, p.ntiles));
    __syncthreads();  // the next tile's staging overwrites this tile's epilogue image in LDS
  }
}

template <int BM, int BN, int WM, int WN, int kEpi, int kAct>
int launch(ConvArgs a, bool im2col, hipStream_t stream) {
  ConvGeom g = a.g;
  g.tiles_n = g.N / BN;
  g.ntiles = (g.M + BM - 1) / BM * g.tiles_n;
  auto kern = conv_kernel<BM, BN, WM, WN, kEpi, kAct, false, false, false>;
  if (a.x2) {
    // The dual source exists for the projection conv3 + shortcut (no residual epilogue).
    if constexpr (kEpi == 0 || kEpi == 1 || kEpi == 6) kern = conv_kernel<BM, BN, WM, WN, kEpi, kAct, false, false, true>;
    else return -1;
  } else if (im2col) {
    kern = conv_kernel<BM, BN, WM, WN, kEpi, kAct, true, false, false>;
  } else if (a.pscale) {
    // The prologue exists for the ResNet-V2 conv1 (BN + ReLU epilogue) only.
    if constexpr (kEpi == 1 && kAct == 1) kern = conv_kernel<BM, BN, WM, WN, kEpi, kAct, false, true, false>;
    else return -1;
  }
  if constexpr (kEpi == 6)
    if (!a.x2) return -1;
  unsigned grid = g.ntiles;
  if (a.max_blocks > 0 && (unsigned)a.max_blocks < grid) grid = a.max_blocks < 8 ? 8u : (unsigned)a.max_blocks / 8u * 8u;
  if (grid > g.ntiles) grid = g.ntiles;
  hipLaunchKernelGGL(kern, dim3(grid), dim3(kThreads), 0, stream, static_cast<const u32x4*>(a.x),
                     static_cast<const u32x4*>(a.x2),
                     static_cast<const u32x4*>(a.w), a.scale, a.shift, static_cast<const u32x4*>(a.r),
                     static_cast<u32x4*>(a.y), static_cast<u32x4*>(a.s), a.pscale, a.pshift, g);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

template <int BM, int BN, int WM, int WN, int kAct>
int by_epi(int epi, const ConvArgs& a, bool im2col, hipStream_t st) {
  switch (epi) {
    case 0: return launch<BM, BN, WM, WN, 0, 0>(a, im2col, st);
    case 1: return launch<BM, BN, WM, WN, 1, kAct>(a, im2col, st);
    case 2: return launch<BM, BN, WM, WN, 2, kAct>(a, im2col, st);
    case 3: return launch<BM, BN, WM, WN, 3, kAct>(a, im2col, st);
    case 4: return launch<BM, BN, WM, WN, 4, kAct>(a, im2col, st);
    case 5: return launch<BM, BN, WM, WN, 5, 0>(a, im2col, st);
    case 6: return launch<BM, BN, WM, WN, 6, kAct>(a, im2col, st);
    default: return -1;
  }
}

template <int BM, int BN, int WM, int WN>
int by_act(int act, int epi, const ConvArgs& a, bool im2col, hipStream_t st) {
  switch (act) {
    case 0: return by_epi<BM, BN, WM, WN, 0>(epi, a, im2col, st);
    case 1: return by_epi<BM, BN, WM, WN, 1>(epi, a, im2col, st);
    case 2: return by_epi<BM, BN, WM, WN, 2>(epi, a, im2col, st);
    default: return -1;
  }
}

// The shared host path of both entry points (x2 == nullptr: single source).
int run_conv(const void* x, const void* w, const float* scale, const float* shift, const void* r, void* y, void* sum,
             const float* pscale, const float* pshift, const void* x2, int nb, int h, int wd, int c, int cout, int kh,
             int kw, int stride, int pad, int c2, int h2, int w2, int stride2, int epi, int act, int max_blocks,
             void* stream) {
  if (!x || !w || !y || nb <= 0 || h <= 0 || wd <= 0 || c <= 0 || cout <= 0 || kh <= 0 || kw <= 0 || stride <= 0 ||
      pad < 0 || pad >= kh || pad >= kw)
    return -1;
  if (c % kBK || cout % 64) return -1;
  if (epi < 0 || epi > 6 || act < 0 || act > 2) return -1;
  if (((epi >= 1 && epi <= 4) || epi == 6) && (!scale || !shift)) return -1;
  if ((pscale == nullptr) != (pshift == nullptr)) return -1;
  if (pscale && (epi != 1 || act != 1 || kh != 1 || kw != 1 || stride != 1 || pad != 0)) return -1;
  if (epi >= 2 && epi <= 5 && !r) return -1;
  if ((epi == 3 || epi == 6) != (sum != nullptr)) return -1;
  if ((epi == 6) && !x2) return -1;
  const int64_t oh = ((int64_t)h + 2 * pad - kh) / stride + 1, ow = ((int64_t)wd + 2 * pad - kw) / stride + 1;
  if (oh <= 0 || ow <= 0 || h + 2 * pad < kh || wd + 2 * pad < kw) return -1;
  if (x2) {  // [x | x2 strided] . [w1 | w2]^T: 1x1 stride-1 source 1, strided 1x1 source 2
    if (kh != 1 || kw != 1 || stride != 1 || pad != 0 || pscale || c2 <= 0 || c2 % kBK || h2 <= 0 || w2 <= 0 ||
        stride2 <= 0 || (h2 - 1) / stride2 + 1 != oh || (w2 - 1) / stride2 + 1 != ow)
      return -1;
    if (epi != 0 && epi != 1 && epi != 6) return -1;
  }
  // Buffer descriptors address with 32-bit offsets below 2^31: the weight must fit, and
  // larger batches run as several launches over groups of whole images.
  const int64_t k = (int64_t)kh * kw * c + (x2 ? c2 : 0), lim = ((int64_t)1 << 31) - 1;
  const int64_t img_x = (int64_t)h * wd * c * 2, img_y = oh * ow * cout * 2;
  const int64_t img_x2 = x2 ? (int64_t)h2 * w2 * c2 * 2 : 0;
  if (k * cout * 2 > lim || img_x > lim || img_y > lim || img_x2 > lim) return -1;
  auto misaligned = [](const void* q) { return q && (reinterpret_cast<uintptr_t>(q) & 15u); };
  if (misaligned(x) || misaligned(w) || misaligned(y) || misaligned(r) || misaligned(sum) || misaligned(scale) ||
      misaligned(shift) || misaligned(pscale) || misaligned(pshift) || misaligned(x2))
    return -1;
  int64_t big = img_x > img_y ? img_x : img_y;
  big = big > img_x2 ? big : img_x2;
  const int64_t per = lim / big;  // images per launch
  const bool im2col = !(kh == 1 && kw == 1 && stride == 1 && pad == 0);
  hipStream_t st = static_cast<hipStream_t>(stream);
  for (int64_t i0 = 0; i0 < nb; i0 += per) {
    const int64_t ni = nb - i0 < per ? nb - i0 : per;
    auto at = [](const void* q, int64_t off) {
      return q ? static_cast<const void*>(static_cast<const char*>(q) + off) : nullptr;
    };
    ConvArgs a{};
    a.pscale = pscale;
    a.pshift = pshift;
    a.max_blocks = max_blocks < 0 ? 0 : max_blocks;
    a.x = at(x, i0 * img_x);
    a.x2 = at(x2, i0 * img_x2);
    a.w = w;
    a.scale = scale;
    a.shift = shift;
    a.r = at(r, i0 * img_y);
    a.y = const_cast<void*>(at(y, i0 * img_y));
    a.s = const_cast<void*>(at(sum, i0 * img_y));
    const int64_t m = ni * oh * ow;
    a.g.M = (unsigned)m;
    a.g.N = (unsigned)cout;
    a.g.K = (unsigned)k;
    a.g.H = (unsigned)h;
    a.g.W = (unsigned)wd;
    a.g.C = (unsigned)c;
    a.g.OH = (unsigned)oh;
    a.g.OW = (unsigned)ow;
    a.g.KW = (unsigned)kw;
    a.g.stride = (unsigned)stride;
    a.g.pad = (unsigned)pad;
    a.g.x_bytes = (unsigned)(ni * img_x);
    a.g.w_bytes = (unsigned)(k * cout * 2);
    if (x2) {
      a.g.C2 = (unsigned)c2;
      a.g.H2 = (unsigned)h2;
      a.g.W2 = (unsigned)w2;
      a.g.stride2 = (unsigned)stride2;
      a.g.x2_bytes = (unsigned)(ni * img_x2);
    }
    // Small-M layers (fewer than two 128-row tiles per CU) use 64-row tiles, so the grid
    // still fills the chip (e.g. ResNet stage 4: 6050 rows x 512 -> 192 vs 380 blocks).
    const int64_t bn = cout % 128 == 0 ? 128 : 64;
    // VGPU_CONV_BM=64|128 forces the row-tile height (measurement).
    static const int force_bm = [] {
      const char* e = getenv("VGPU_CONV_BM");
      return e ? atoi(e) : 0;
    }();
    const bool small_m = force_bm ? force_bm == 64 : (m + 127) / 128 * (cout / bn) < 512;
    int rc;
    if (bn == 128)
      rc = small_m ? by_act<64, 128, 2, 2>(act, epi, a, im2col, st) : by_act<128, 128, 2, 2>(act, epi, a, im2col, st);
    else
      rc = small_m ? by_act<64, 64, 2, 2>(act, epi, a, im2col, st) : by_act<128, 64, 4, 1>(act, epi, a, im2col, st);
    if (rc) return rc;
  }
  return 0;
}

}  // namespace

extern "C" {

// y[Nb, OH, OW, Cout] = epilogue(conv(x[Nb, H, W, C], w[Cout, KH, KW, C])), bf16 NHWC,
// fp32 accumulation, OH = (H + 2 pad - KH) / stride + 1 (same for OW). epi: 0 plain,
// 1 act(acc*scale+shift), 2 act((acc+r)*scale+shift), 3 as 2 and sum = acc + r,
// 4 act(acc*scale + shift + r), 5 acc + r. act: 0 none, 1 relu, 2 relu6. scale/shift:
// fp32[Cout]. pscale/pshift (optional, fp32[C], 1x1 stride-1 with epi 1 + relu only): the
// input is read as relu(x * pscale + pshift). max_blocks > 0 caps the grid (persistent
// blocks; rounded down to a multiple of 8). Returns 0 on success, -1 on bad arguments,
// -2 on launch failure.
int vgpu_conv_nhwc_bf16(const void* x, const void* w, const float* scale, const float* shift, const void* r, void* y,
                        void* sum, const float* pscale, const float* pshift, int nb, int h, int wd, int c, int cout,
                        int kh, int kw, int stride, int pad, int epi, int act, int max_blocks, void* stream) {
  if (epi > 5) return -1;
  return run_conv(x, w, scale, shift, r, y, sum, pscale, pshift, nullptr, nb, h, wd, c, cout, kh, kw, stride, pad, 0, 0,
                  0, 0, epi, act, max_blocks, stream);
}

// Projection block: y[Nb, H, W, Cout] = epilogue(x[Nb, H, W, C] . w1^T + x2[:, ::s2, ::s2, :] . w2^T)
// with w = [Cout][C + C2] (w1 | w2 along K) and x2 [Nb, H2, W2, C2], (H2 - 1) / s2 + 1 == H
// (same for W). epi: 0 plain, 1 act(acc*scale+shift), 6 as 1 and sum = acc. Returns as
// vgpu_conv_nhwc_bf16.
int vgpu_conv_dual_bf16(const void* x, const void* x2, const void* w, const float* scale, const float* shift, void* y,
                        void* sum, int nb, int h, int wd, int c, int c2, int h2, int w2, int stride2, int cout, int epi,
                        int act, int max_blocks, void* stream) {
  if (!x2) return -1;
  return run_conv(x, w, scale, shift, nullptr, y, sum, nullptr, nullptr, x2, nb, h, wd, c, cout, 1, 1, 1, 0, c2, h2, w2,
                  stride2, epi, act, max_blocks, stream);
}

// 1x1 / stride-1 convolution over M pixels: y[M, N] = epilogue(x[M, K] . w[N, K]^T).
int vgpu_conv1x1_bf16(const void* x, const void* w, const float* scale, const float* shift, const void* r, void* y,
                      void* sum, int64_t M, int N, int K, int epi, int act, void* stream) {
  if (M <= 0 || M >= ((int64_t)1 << 31)) return -1;
  return vgpu_conv_nhwc_bf16(x, w, scale, shift, r, y, sum, nullptr, nullptr, (int)M, 1, 1, K, N, 1, 1, 1, 0, epi, act,
                             0, stream);
}

}  // extern "C"
