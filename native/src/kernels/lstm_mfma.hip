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
__device__ __forceinline__ float sigmoid(float x) { return 1.0f / (1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_fast(float x) { return 2.0f * sigmoid(2.0f * x) - 1.0f; }

// gx: [B, T, 128, 4] bf16 (gate order i, f, g, o), whh: [512, 128] bf16 (PyTorch
// weight_hh_l0, rows i|f|g|o), h0/c0: [B, 128] fp32 or null (zeros), hT/cT: [B, 128] fp32
// (cT may be null).
__global__ void __launch_bounds__(kThreads) lstm_kernel(const u32x2* __restrict__ gx, const u32x4* __restrict__ whh,
                                                       const float* __restrict__ h0, const float* __restrict__ c0,
                                                       float* __restrict__ hT, float* __restrict__ cT, unsigned B,
                                                       unsigned T) {
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
  // Gate-input addresses (row clamped to a valid one past the batch; never stored).
  const u32x2* gsrc[2][4];
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) {
      unsigned b = b0 + 4u * q4 + r;
      b = b < B ? b : B - 1u;
      const unsigned u = wave * kUnitsPerWave + 16u * jj + l16;
      gsrc[jj][r] = gx + (size_t)b * T * kH + u;  // + t * kH per step
    }
  u32x2 gcur[2][4];
#pragma unroll
  for (int jj = 0; jj < 2; jj++)
#pragma unroll
    for (int r = 0; r < 4; r++) gcur[jj][r] = gsrc[jj][r][0];
  __syncthreads();

  for (unsigned t = 0; t < T; t++) {
    const unsigned cur = t & 1u;
    // Next step's gate inputs, in flight under this step's MFMAs.
    u32x2 gnext[2][4];
    const unsigned tn = t + 1 < T ? t + 1 : t;
#pragma unroll
    for (int jj = 0; jj < 2; jj++)
#pragma unroll
      for (int r = 0; r < 4; r++) gnext[jj][r] = gsrc[jj][r][(size_t)tn * kH];

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
        const float cn = sigmoid(gf) * c[jj][r] + sigmoid(gi) * tanh_fast(gg);
        c[jj][r] = cn;
        h[jj][r] = sigmoid(go) * tanh_fast(cn);
        hbuf[cur ^ 1u][4u * q4 + r][wave * kUnitsPerWave + 16u * jj + l16] = to_bf16(h[jj][r]);
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

}  // namespace

extern "C" {

// Runs the recurrence of a 128-unit LSTM layer over T steps for B sequences (see
// lstm_kernel for the layouts). Returns 0 on success, -1 on bad arguments, -2 on launch
// failure.
int vgpu_lstm_seq_bf16(const void* gx, const void* whh, const float* h0, const float* c0, float* hT, float* cT,
                       int batch, int steps, int hidden, void* stream) {
  if (!gx || !whh || !hT || batch <= 0 || steps <= 0 || hidden != kH) return -1;
  if ((int64_t)batch * steps * kH * 4 >= ((int64_t)1 << 34)) return -1;
  auto misaligned = [](const void* p, uintptr_t a) { return p && (reinterpret_cast<uintptr_t>(p) & (a - 1)); };
  if (misaligned(gx, 8) || misaligned(whh, 16) || misaligned(h0, 4) || misaligned(c0, 4) || misaligned(hT, 4) ||
      misaligned(cT, 4))
    return -1;
  const unsigned blocks = (unsigned)((batch + kRows - 1) / kRows);
  hipLaunchKernelGGL(lstm_kernel, dim3(blocks), dim3(kThreads), 0, static_cast<hipStream_t>(stream),
                     static_cast<const u32x2*>(gx), static_cast<const u32x4*>(whh), h0, c0, hT, cT, (unsigned)batch,
                     (unsigned)steps);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // extern "C"
