// Single-layer LSTM recurrence (hidden 128) on gfx950 matrix cores, the whole sequence in
// one persistent kernel: the in-pod LSTM workloads (ai-benchmark 5.1/5.2: 1024 steps, 300
// features, 128 hidden units, batch 100).
//
// Run through the library, every time step is its own handful of launches (a small GEMM
// for h . W_hh^T, the gate nonlinearities, the cell update): 1024 steps are launch- and
// latency-bound (profiles/r1k: 46 ms eager, 13.5 ms replayed from a HIP graph for a batch
// whose arithmetic is ~30 GFLOP). Here:
//
//   * the input projection x . W_ih^T + b for all steps is one library GEMM beforehand,
//     with W_ih's rows permuted so the four gates of one hidden unit are adjacent
//     (gx[b, t, unit, gate], one 8-byte load per (row, unit) per step);
//   * one workgroup owns 16 batch rows for the whole sequence; its 4 wave64s each own 32
//     hidden units, i.e. 128 gate columns (4 gates x 32 units) of W_hh^T, held in
//     registers as MFMA B fragments for all 1024 steps (128 VGPRs);
//   * per step each wave runs 32 v_mfma_f32_16x16x32_bf16 (h_t [16 x 128] from LDS as the
//     A operand), and because a lane's four gate fragments share (row, unit), the cell
//     update c = f c + i g, h = o tanh(c) is lane-local with c kept in registers;
//   * h_{t+1} goes to the other half of a double-buffered 4 KB LDS image: one barrier per
//     step. The next step's gate inputs are loaded while the current step computes.
//
// Numerics: bf16 operands, fp32 accumulation and fp32 cell state; h is rounded to bf16
// each step (it is the next MFMA's operand), as a bf16 library LSTM stores it.
// C ABI (ctypes): pointers are device pointers, `stream` a hipStream_t.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

using u32x2 = unsigned int __attribute__((ext_vector_type(2)));
using u32x4 = unsigned int __attribute__((ext_vector_type(4)));
using f32x4 = float __attribute__((ext_vector_type(4)));
using bf16x8 = __bf16 __attribute__((ext_vector_type(8)));

constexpr int kH = 128;        // hidden units
constexpr int kRows = 16;      // batch rows per workgroup (one MFMA M fragment)
constexpr int kWaves = 4;      // 32 hidden units per wave
constexpr int kUnitsPerWave = kH / kWaves;
constexpr int kThreads = kWaves * 64;

__device__ __forceinline__ float bf_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }
__device__ __forceinline__ unsigned short to_bf16(float f) { return __bfloat16_as_ushort(__float2bfloat16(f)); }
// Raw v_exp_f32 + v_rcp_f32 (1 ulp): an IEEE division here expanded to ~10 VALU
// instructions per gate and made the serial step VALU-bound (profiles/r1ax).
__device__ __forceinline__ float sigmoid(float x) {
  return __builtin_amdgcn_rcpf(1.0f + __builtin_amdgcn_exp2f(x * -1.4426950408889634f));
}
__device__ __forceinline__ float tanh_fast(float x) { return 2.0f * sigmoid(2.0f * x) - 1.0f; }

// Raw buffer descriptor over [p, p + bytes) (bytes < 2^31, checked on the host). Per-step
// traffic goes through these: a lane's voffset is fixed for the whole sequence and the
// step is the wave-uniform soffset, so there is no 64-bit address arithmetic in the serial
// loop, and a row past the batch gets voffset kOOB: its stores are dropped by the range
// check instead of branched around.
__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  const uint64_t a = reinterpret_cast<uint64_t>(p);
  const uint64_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
  const uint64_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
  return __builtin_amdgcn_make_buffer_rsrc(reinterpret_cast<void*>((hi << 32) | lo), (short)0,
                                           (int)__builtin_amdgcn_readfirstlane(bytes), 0x00020000);
}
constexpr unsigned kOOB = 0x80000000u;
// A per-step soffset made provably wave-uniform (else the buffer op is wrapped in a
// readfirstlane waterfall loop).
__device__ __forceinline__ unsigned uni(unsigned v) { return (unsigned)__builtin_amdgcn_readfirstlane((int)v); }

// gx: [B, T, 128, 4] bf16 (gate order i, f, g, o), whh: [512, 128] bf16 (PyTorch
// weight_hh_l0, rows i|f|g|o), h0/c0: [B, 128] fp32 or null (zeros), hT/cT: [B, 128] fp32
// (cT may be null). kStash (training): also writes, per step, the gate activations
// act[B, T, 128] float4 (i, f, g, o), the cell state cs[B, T, 128] fp32 and h hs[B, T, 128]
// bf16 (the value the next step's MFMA used) for the backward recurrence.
template <bool kStash>
__global__ void __launch_bounds__(kThreads) lstm_kernel(const u32x2* __restrict__ gx, const u32x4* __restrict__ whh,
                                                       const float* __restrict__ h0, const float* __restrict__ c0,
                                                       float* __restrict__ hT, float* __restrict__ cT,
                                                       float4* __restrict__ act, float* __restrict__ cs,
                                                       unsigned short* __restrict__ hs, unsigned B, unsigned T) {
  const unsigned cells = B * T * kH;  // < 2^27 (host check): every byte range below < 2^31
  const __amdgpu_buffer_rsrc_t gxr = make_rsrc(gx, cells * 8u);
  const __amdgpu_buffer_rsrc_t actr = make_rsrc(kStash ? static_cast<const void*>(act) : gx, kStash ? cells * 16u : 0u);
  const __amdgpu_buffer_rsrc_t csr = make_rsrc(kStash ? static_cast<const void*>(cs) : gx, kStash ? cells * 4u : 0u);
  const __amdgpu_buffer_rsrc_t hsr = make_rsrc(kStash ? static_cast<const void*>(hs) : gx, kStash ? cells * 2u : 0u);
  __shared__ __attribute__((aligned(16))) unsigned short hbuf[2][kRows][kH];
  const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const unsigned l16 = lane & 15u, q4 = lane >> 4;  // q4: k-quarter for A/B, row group for C/D
  const unsigned b0 = blockIdx.x * kRows;

  // W_hh^T fragments: N-fragment j (0..7) = gate j/2, units 32 wave + 16 (j%2) + 0..15;
  // B[k][n] = W_hh[gate*128 + unit][k]; lane holds k = 32 kk + 8 q4 + 0..7 of column l16.
  bf16x8 wf[8][4];
#pragma unroll
  for (int j = 0; j < 8; j++) {
    const unsigned row = (j >> 1) * kH + wave * kUnitsPerWave + (j & 1) * 16u + l16;
#pragma unroll
    for (int kk = 0; kk < 4; kk++) wf[j][kk] = __builtin_bit_cast(bf16x8, whh[row * (kH / 8) + kk * 4 + q4]);
  }

  // This lane's cells: rows 4 q4 + r, units 32 wave + 16 jj + l16.
  float c[2][4], h[2][4];
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned b = b0 + 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
      const bool ok = b < B;
      c[jj][r] = (ok && c0) ? c0[(size_t)b * kH + u] : 0.f;
      h[jj][r] = (ok && h0) ? h0[(size_t)b * kH + u] : 0.f;
      hbuf[0][4u * q4 + r][u] = to_bf16(h[jj][r]);
    }
  // Cell index of (row, unit) at step 0 (+ t * kH per step); gate inputs of a row past the
  // batch are read from a clamped valid row (never stored), its stash stores are dropped.
  unsigned e_ld[2][4], e_st[2][4];
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned b = b0 + 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
      e_ld[jj][r] = ((b < B ? b : B - 1u) * T) * kH + u;
      e_st[jj][r] = b < B ? (b * T) * kH + u : kOOB;
    }
  auto ld_gx = [&](int jj, int r, unsigned t) {
    const auto v = __builtin_amdgcn_raw_buffer_load_b64(gxr, e_ld[jj][r] * 8u, uni(t * (kH * 8u)), 0);
    return u32x2{v[0], v[1]};
  };
  u32x2 gcur[2][4];
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) gcur[jj][r] = ld_gx(jj, r, 0);
  __syncthreads();

  for (unsigned t = 0; t < T; t++) {
    const unsigned cur = t & 1u;
    // Next step's gate inputs, in flight under this step's MFMAs.
    u32x2 gnext[2][4];
    const unsigned tn = t + 1 < T ? t + 1 : t;
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) gnext[jj][r] = ld_gx(jj, r, tn);

    f32x4 acc[8];
#pragma unroll
    for (int j = 0; j < 8; j++) acc[j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kk = 0; kk < 4; kk++) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(&hbuf[cur][l16][kk * 32 + q4 * 8]));
#pragma unroll
      for (int j = 0; j < 8; j++) acc[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[j][kk], acc[j], 0, 0, 0);
    }
    // C/D: column l16 (unit within the fragment), row 4 q4 + r (batch row).
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const u32x2 g = gcur[jj][r];  // (i, f) in g.x, (g, o) in g.y, bf16 pairs
        const float gi = acc[0 + jj][r] + bf_lo(g.x);
        const float gf = acc[2 + jj][r] + bf_hi(g.x);
        const float gg = acc[4 + jj][r] + bf_lo(g.y);
        const float go = acc[6 + jj][r] + bf_hi(g.y);
        const float si = sigmoid(gi), sf = sigmoid(gf), tg = tanh_fast(gg), so = sigmoid(go);
        const float cn = sf * c[jj][r] + si * tg;
        c[jj][r] = cn;
        h[jj][r] = so * tanh_fast(cn);
        const unsigned short hb = to_bf16(h[jj][r]);
        hbuf[cur ^ 1u][4u * q4 + r][wave * kUnitsPerWave + 16u * jj + l16] = hb;
        if constexpr (kStash) {
          const unsigned e = e_st[jj][r];  // kOOB (dropped) past the batch
          using u32x4_t = unsigned int __attribute__((ext_vector_type(4)));
          const u32x4_t a4 = {__float_as_uint(si), __float_as_uint(sf), __float_as_uint(tg), __float_as_uint(so)};
          __builtin_amdgcn_raw_buffer_store_b128(a4, actr, e == kOOB ? kOOB : e * 16u, uni(t * (kH * 16u)), 0);
          __builtin_amdgcn_raw_buffer_store_b32(__float_as_uint(cn), csr, e == kOOB ? kOOB : e * 4u, uni(t * (kH * 4u)), 0);
          __builtin_amdgcn_raw_buffer_store_b16(hb, hsr, e == kOOB ? kOOB : e * 2u, uni(t * (kH * 2u)), 0);
        }
      }
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) gcur[jj][r] = gnext[jj][r];
    __syncthreads();
  }

#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned b = b0 + 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
      if (b >= B) continue;
      hT[(size_t)b * kH + u] = h[jj][r];
      if (cT) cT[(size_t)b * kH + u] = c[jj][r];
    }
}

// Backward recurrence (BPTT) of the layer above, for a loss on h_T only (the sentiment
// model reads the last hidden state), over the forward's stash. Per step, lane-local like
// the forward (a lane owns cells (row 4 q4 + r, unit 32 wave + 16 jj + l16)):
//   dc += dh o (1 - tanh(c)^2);  dz_o = dh tanh(c) o (1 - o);  dz_i = dc g i (1 - i);
//   dz_g = dc i (1 - g^2);  dz_f = dc c_{t-1} f (1 - f);  dc = dc f
// then dh_{t-1} = dz_t . W_hh ([16 x 512] . [512 x 128]) on the matrix cores: W_hh (as
// whhT = W_hh^T [128, 512], row n = hidden unit n) in registers as B fragments for the
// whole sequence (2 N-fragments x 16 K-chunks per wave, 128 VGPRs), dz_t through a
// double-buffered LDS image (rows padded by 16 B: conflict-free fragment reads).
// dz is also written out ([B, T, 512] bf16, columns gate-major i|f|g|o like PyTorch's
// weight rows) for the weight-gradient GEMMs. dh0/dc0: gradients of the initial state.
// Its per-step traffic stays on plain global pointers: moving it to buffer descriptors
// like the forward's pushed the kernel to 256 VGPRs, the compiler then serialised the
// next step's loads (vmcnt(0) after each) and the kernel ran 2x slower (profiles/r1ay).
constexpr int kG = 4 * kH;       // gate columns
constexpr int kZStride = kG + 8;  // bf16 per LDS row of dz

__global__ void __launch_bounds__(kThreads) lstm_bwd_kernel(const u32x4* __restrict__ whhT,
                                                           const float4* __restrict__ act,
                                                           const float* __restrict__ cs, const float* __restrict__ c0,
                                                           const float* __restrict__ dhT, const float* __restrict__ dcT,
                                                           unsigned short* __restrict__ dz, float* __restrict__ dh0,
                                                           float* __restrict__ dc0, unsigned B, unsigned T) {
  __shared__ __attribute__((aligned(16))) unsigned short zbuf[2][kRows][kZStride];
  const unsigned tid = threadIdx.x, lane = tid & 63u, wave = tid >> 6;
  const unsigned l16 = lane & 15u, q4 = lane >> 4;
  const unsigned b0 = blockIdx.x * kRows;

  // B[k][n] = W_hh[k][n] = whhT[n][k]: N-fragment jj = units 32 wave + 16 jj + 0..15;
  // lane holds k = 32 kk + 8 q4 + 0..7 of column l16.
  bf16x8 wf[2][16];
#pragma unroll
  for (int jj = 0; jj < 2; jj++) {
    const unsigned n = wave * kUnitsPerWave + jj * 16u + l16;
#pragma unroll
    for (int kk = 0; kk < 16; kk++) wf[jj][kk] = __builtin_bit_cast(bf16x8, whhT[n * (kG / 8) + kk * 4 + q4]);
  }

  float dh[2][4], dc[2][4], ccur[2][4];
  size_t base[2][4];
  bool ok[2][4];
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned b = b0 + 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
      ok[jj][r] = b < B;
      const unsigned bc = b < B ? b : B - 1u;  // clamped row: loads stay in bounds, never stored
      base[jj][r] = (size_t)bc * T * kH + u;   // + t * kH per step
      dh[jj][r] = ok[jj][r] ? dhT[(size_t)b * kH + u] : 0.f;
      dc[jj][r] = (ok[jj][r] && dcT) ? dcT[(size_t)b * kH + u] : 0.f;
      ccur[jj][r] = cs[base[jj][r] + (size_t)(T - 1) * kH];
    }
  // Step t needs act_t, c_t (carried) and c_{t-1}; step t's loads for t - 1 go out first.
  float4 acur[2][4];
  float cprev[2][4];
  auto load_prev = [&](unsigned t, int jj, int r) -> float {  // c_{t-1}
    if (t > 0) return cs[base[jj][r] + (size_t)(t - 1) * kH];
    const unsigned b = b0 + 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
    return (ok[jj][r] && c0) ? c0[(size_t)b * kH + u] : 0.f;
  };
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      acur[jj][r] = act[base[jj][r] + (size_t)(T - 1) * kH];
      cprev[jj][r] = load_prev(T - 1, jj, r);
    }

  for (unsigned s = 0; s < T; s++) {
    const unsigned t = T - 1u - s, cur = s & 1u;
    const unsigned tn = t > 0 ? t - 1u : 0u;
    float4 anext[2][4];
    float cpn[2][4];
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        anext[jj][r] = act[base[jj][r] + (size_t)tn * kH];
        cpn[jj][r] = load_prev(tn, jj, r);
      }
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) {
        const float4 a = acur[jj][r];  // i, f, g, o
        const float tc = tanh_fast(ccur[jj][r]);
        const float d = dh[jj][r];
        const float dct = dc[jj][r] + d * a.w * (1.f - tc * tc);
        const float zo = d * tc * a.w * (1.f - a.w);
        const float zi = dct * a.z * a.x * (1.f - a.x);
        const float zg = dct * a.x * (1.f - a.z * a.z);
        const float zf = dct * cprev[jj][r] * a.y * (1.f - a.y);
        dc[jj][r] = dct * a.y;
        const unsigned row = 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
        const unsigned short bi = to_bf16(zi), bf = to_bf16(zf), bg = to_bf16(zg), bo = to_bf16(zo);
        zbuf[cur][row][u] = bi;
        zbuf[cur][row][kH + u] = bf;
        zbuf[cur][row][2 * kH + u] = bg;
        zbuf[cur][row][3 * kH + u] = bo;
        if (ok[jj][r]) {
          unsigned short* zr = dz + ((size_t)(b0 + row) * T + t) * kG + u;
          zr[0] = bi;
          zr[kH] = bf;
          zr[2 * kH] = bg;
          zr[3 * kH] = bo;
        }
        ccur[jj][r] = cprev[jj][r];
        acur[jj][r] = anext[jj][r];
        cprev[jj][r] = cpn[jj][r];
      }
    __syncthreads();  // dz_t complete in LDS; the other buffer's readers (step s - 1) are done
    f32x4 acc[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
#pragma unroll
    for (int kk = 0; kk < 16; kk++) {
      const bf16x8 a = __builtin_bit_cast(bf16x8, *reinterpret_cast<const u32x4*>(&zbuf[cur][l16][kk * 32 + q4 * 8]));
      acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[0][kk], acc[0], 0, 0, 0);
      acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(a, wf[1][kk], acc[1], 0, 0, 0);
    }
    // C/D: column l16 (unit within fragment jj), row 4 q4 + r: exactly this lane's cells.
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) dh[jj][r] = acc[jj][r];
  }

#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      const unsigned b = b0 + 4u * q4 + r, u = wave * kUnitsPerWave + 16u * jj + l16;
      if (!ok[jj][r]) continue;
      if (dh0) dh0[(size_t)b * kH + u] = dh[jj][r];
      if (dc0) dc0[(size_t)b * kH + u] = dc[jj][r];
    }
}

}  // namespace

extern "C" {

// Runs the recurrence of a 128-unit LSTM layer over T steps for B sequences (see
// lstm_kernel for the layouts). Returns 0 on success, -1 on bad arguments, -2 on launch
// failure.
int vgpu_lstm_seq_bf16(const void* gx, const void* whh, const float* h0, const float* c0, float* hT, float* cT,
                       int batch, int steps, int hidden, void* stream) {
  if (!gx || !whh || !hT || batch <= 0 || steps <= 0 || hidden != kH) return -1;
  if ((int64_t)batch * steps * kH * 8 >= ((int64_t)1 << 31)) return -1;  // buffer-descriptor range
  auto misaligned = [](const void* p, uintptr_t a) { return p && (reinterpret_cast<uintptr_t>(p) & (a - 1)); };
  if (misaligned(gx, 8) || misaligned(whh, 16) || misaligned(h0, 4) || misaligned(c0, 4) || misaligned(hT, 4) ||
      misaligned(cT, 4))
    return -1;
  const unsigned blocks = (unsigned)((batch + kRows - 1) / kRows);
  hipLaunchKernelGGL(lstm_kernel<false>, dim3(blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x2*>(gx), static_cast<const u32x4*>(whh), h0, c0, hT, cT, nullptr, nullptr,
                     nullptr, (unsigned)batch, (unsigned)steps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Training forward: vgpu_lstm_seq_bf16 plus the stash of the backward recurrence:
// act [B, T, 128, 4] fp32 (sigmoid i, sigmoid f, tanh g, sigmoid o), cs [B, T, 128] fp32
// (c_t), hs [B, T, 128] bf16 (h_t).
int vgpu_lstm_seq_train_bf16(const void* gx, const void* whh, const float* h0, const float* c0, float* hT,
                             float* cT, float* act, float* cs, void* hs, int batch, int steps, int hidden,
                             void* stream) {
  if (!gx || !whh || !hT || !act || !cs || !hs || batch <= 0 || steps <= 0 || hidden != kH) return -1;
  if ((int64_t)batch * steps * kH * 16 >= ((int64_t)1 << 31)) return -1;  // buffer-descriptor ranges
  auto misaligned = [](const void* p, uintptr_t a) { return p && (reinterpret_cast<uintptr_t>(p) & (a - 1)); };
  if (misaligned(gx, 8) || misaligned(whh, 16) || misaligned(h0, 4) || misaligned(c0, 4) || misaligned(hT, 4) ||
      misaligned(cT, 4) || misaligned(act, 16) || misaligned(cs, 4) || misaligned(hs, 2))
    return -1;
  const unsigned blocks = (unsigned)((batch + kRows - 1) / kRows);
  hipLaunchKernelGGL(lstm_kernel<true>, dim3(blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x2*>(gx), static_cast<const u32x4*>(whh), h0, c0, hT, cT,
                     reinterpret_cast<float4*>(act), cs, static_cast<unsigned short*>(hs), (unsigned)batch,
                     (unsigned)steps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

// Backward recurrence for a loss on h_T: whhT = W_hh^T [128, 512] bf16, act/cs the
// training forward's stash, c0 [B, 128] fp32 or null, dhT [B, 128] fp32, dcT [B, 128] fp32
// or null. Writes dz [B, T, 512] bf16 (pre-activation gate gradients, columns i|f|g|o) and,
// when non-null, dh0/dc0 [B, 128] fp32.
int vgpu_lstm_seq_bwd_bf16(const void* whhT, const float* act, const float* cs, const float* c0, const float* dhT,
                           const float* dcT, void* dz, float* dh0, float* dc0, int batch, int steps, int hidden,
                           void* stream) {
  if (!whhT || !act || !cs || !dhT || !dz || batch <= 0 || steps <= 0 || hidden != kH) return -1;
  if ((int64_t)batch * steps * kH * 16 >= ((int64_t)1 << 31)) return -1;  // buffer-descriptor ranges
  auto misaligned = [](const void* p, uintptr_t a) { return p && (reinterpret_cast<uintptr_t>(p) & (a - 1)); };
  if (misaligned(whhT, 16) || misaligned(act, 16) || misaligned(cs, 4) || misaligned(c0, 4) || misaligned(dhT, 4) ||
      misaligned(dcT, 4) || misaligned(dz, 2) || misaligned(dh0, 4) || misaligned(dc0, 4))
    return -1;
  const unsigned blocks = (unsigned)((batch + kRows - 1) / kRows);
  hipLaunchKernelGGL(lstm_bwd_kernel, dim3(blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x4*>(whhT), reinterpret_cast<const float4*>(act), cs, c0, dhT, dcT,
                     static_cast<unsigned short*>(dz), dh0, dc0, (unsigned)batch, (unsigned)steps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
