// Fused inference epilogues for the in-pod benchmark workloads (gfx950, bf16, NHWC).
//
//   y   = act(x * scale[c] + shift[c])                      (BN(eval) + ReLU)
//   s   = x + r ;  y = act(s * scale[c] + shift[c])          (residual add + next BN + ReLU;
//                                                             pre-activation ResNet blocks)
//   y   = act(x * scale[c] + shift[c] + r)                  (BN of the last conv + residual;
//                                                             MobileNet-V2 / post-activation)
//
// In a pre-activation ResNet every block boundary is "add the shortcut, then the next
// block's BN + ReLU", and every conv inside a block is followed by BN + ReLU. Eager
// PyTorch runs each of those as 3-5 separate passes over the activation (BN transform,
// clamp, add, the bf16<->f32 copies and the inv-std kernel: ~37 % of the ResNet-V2-50
// inference step on MI355X, profiles/r1a_resnet50_inf_vgpu.md). These kernels do one
// pass: 16-byte (8 x bf16) loads/stores per lane, fp32 math, per-channel scale/shift
// from the L1/L2-resident parameter vectors, round-to-nearest-even back to bf16
// (v_cvt_pk_bf16_f32). Memory bound by design: bytes moved = inputs + outputs once.
//
// C ABI (ctypes): pointers are device pointers, `stream` a hipStream_t.
#include <hip/hip_bf16.h>
#include <hip/hip_runtime.h>

#include <cstdint>

namespace {

using u32x4 = unsigned int __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf_lo(unsigned v) { return __uint_as_float(v << 16); }
__device__ __forceinline__ float bf_hi(unsigned v) { return __uint_as_float(v & 0xffff0000u); }

// Two floats -> packed bf16 pair (round to nearest even) in one v_cvt_pk_bf16_f32.
__device__ __forceinline__ unsigned pack_bf16(float lo, float hi) {
  using f32x2_t = float __attribute__((ext_vector_type(2)));
  using bf16x2_t = __bf16 __attribute__((ext_vector_type(2)));
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{lo, hi}, bf16x2_t));
}

struct Params8 {
  float sc[8];
  float sh[8];
};

__device__ __forceinline__ Params8 load_params(const float* __restrict__ scale, const float* __restrict__ shift,
                                               unsigned c0) {
  Params8 p;
  const float4 s0 = *reinterpret_cast<const float4*>(scale + c0);
  const float4 s1 = *reinterpret_cast<const float4*>(scale + c0 + 4);
  const float4 t0 = *reinterpret_cast<const float4*>(shift + c0);
  const float4 t1 = *reinterpret_cast<const float4*>(shift + c0 + 4);
  p.sc[0] = s0.x; p.sc[1] = s0.y; p.sc[2] = s0.z; p.sc[3] = s0.w;
  p.sc[4] = s1.x; p.sc[5] = s1.y; p.sc[6] = s1.z; p.sc[7] = s1.w;
  p.sh[0] = t0.x; p.sh[1] = t0.y; p.sh[2] = t0.z; p.sh[3] = t0.w;
  p.sh[4] = t1.x; p.sh[5] = t1.y; p.sh[6] = t1.z; p.sh[7] = t1.w;
  return p;
}

// kAdd: 0 no residual, 1 residual added before the affine, 2 residual added after it.
template <int kAdd, bool kWriteSum, int kAct>
__device__ __forceinline__ void apply8(const u32x4& xv, const u32x4& rv, const Params8& p, u32x4* yv, u32x4* sv) {
  float v[8];
#pragma unroll
  for (int k = 0; k < 4; k++) {
    v[2 * k] = bf_lo(xv[k]);
    v[2 * k + 1] = bf_hi(xv[k]);
  }
  if constexpr (kAdd == 1) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      v[2 * k] += bf_lo(rv[k]);
      v[2 * k + 1] += bf_hi(rv[k]);
    }
    if constexpr (kWriteSum) {
#pragma unroll
      for (int k = 0; k < 4; k++) (*sv)[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
    }
  }
  float post[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  if constexpr (kAdd == 2) {
#pragma unroll
    for (int k = 0; k < 4; k++) {
      post[2 * k] = bf_lo(rv[k]);
      post[2 * k + 1] = bf_hi(rv[k]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; j++) {
    float o = fmaf(v[j], p.sc[j], p.sh[j]);
    if constexpr (kAdd == 2) o += post[j];
    if constexpr (kAct == 1) o = fmaxf(o, 0.0f);
    if constexpr (kAct == 2) o = fminf(fmaxf(o, 0.0f), 6.0f);
    v[j] = o;
  }
#pragma unroll
  for (int k = 0; k < 4; k++) (*yv)[k] = pack_bf16(v[2 * k], v[2 * k + 1]);
}

// Each lane handles two 16-byte vectors per iteration (ILP: both loads in flight before
// the math). nvec < 2^31 is checked on the host, so indexing stays 32-bit.
//
// kHoist: the grid stride (blocks * 256) is a multiple of C/8, so a lane's channel group
// never changes across iterations - its 8 scales and 8 shifts are loaded once into
// registers instead of 64 parameter bytes per 16 activation bytes re-read from L1 on
// every iteration. Holds for every power-of-two C <= 2048 (all ResNet widths); other
// widths (MobileNet's 96/144/...) take the per-vector path.
template <int kAdd, bool kWriteSum, int kAct, bool kHoist>
__global__ void __launch_bounds__(256) bn_act_kernel(const u32x4* __restrict__ x, const u32x4* __restrict__ r,
                                                     const float* __restrict__ scale,
                                                     const float* __restrict__ shift, u32x4* __restrict__ y,
                                                     u32x4* __restrict__ sum, unsigned nvec, unsigned cvec) {
  const unsigned stride = gridDim.x * 256u;
  unsigned i = blockIdx.x * 256u + threadIdx.x;
  Params8 ph;
  if constexpr (kHoist) ph = load_params(scale, shift, (i % cvec) * 8u);
  for (; i + stride < nvec; i += 2 * stride) {
    const unsigned j = i + stride;
    u32x4 xa = __builtin_nontemporal_load(&x[i]);
    u32x4 xb = __builtin_nontemporal_load(&x[j]);
    u32x4 ra{}, rb{};
    if constexpr (kAdd) {
      ra = __builtin_nontemporal_load(&r[i]);
      rb = __builtin_nontemporal_load(&r[j]);
    }
    u32x4 ya, yb, sa, sb;
    if constexpr (kHoist) {
      apply8<kAdd, kWriteSum, kAct>(xa, ra, ph, &ya, &sa);
      apply8<kAdd, kWriteSum, kAct>(xb, rb, ph, &yb, &sb);
    } else {
      apply8<kAdd, kWriteSum, kAct>(xa, ra, load_params(scale, shift, (i % cvec) * 8u), &ya, &sa);
      apply8<kAdd, kWriteSum, kAct>(xb, rb, load_params(scale, shift, (j % cvec) * 8u), &yb, &sb);
    }
    y[i] = ya;
    y[j] = yb;
    if constexpr (kWriteSum) {
      sum[i] = sa;
      sum[j] = sb;
    }
  }
  if (i < nvec) {
    u32x4 xa = __builtin_nontemporal_load(&x[i]);
    u32x4 ra{};
    if constexpr (kAdd) ra = __builtin_nontemporal_load(&r[i]);
    u32x4 ya, sa;
    if constexpr (kHoist) apply8<kAdd, kWriteSum, kAct>(xa, ra, ph, &ya, &sa);
    else apply8<kAdd, kWriteSum, kAct>(xa, ra, load_params(scale, shift, (i % cvec) * 8u), &ya, &sa);
    y[i] = ya;
    if constexpr (kWriteSum) sum[i] = sa;
  }
}

int g_block_cap = 0;  // vgpu_bn_act_set_block_cap

template <int kAdd, bool kWriteSum, int kAct>
void launch(const void* x, const void* r, const float* scale, const float* shift, void* y, void* sum, unsigned nvec,
            unsigned cvec, hipStream_t stream) {
  // Enough waves to cover HBM latency on 256 CUs (>= 8 blocks/CU), capped so every
  // lane does at least a couple of iterations on large tensors.
  unsigned blocks = (nvec + 511u) / 512u;
  if (blocks > 256u * 16u) blocks = 256u * 16u;
  // Inside a CU-masked vGPU: no more blocks than the slice holds at once (one dispatch
  // round, profiles/r1z); the grid-stride loop covers the rest.
  if (g_block_cap > 0 && blocks > (unsigned)g_block_cap) blocks = (unsigned)g_block_cap;
  if (blocks < 1u) blocks = 1u;
  if (256u % cvec == 0u) {  // stride = blocks * 256 is then a multiple of cvec
    hipLaunchKernelGGL((bn_act_kernel<kAdd, kWriteSum, kAct, true>), dim3(blocks), dim3(256), 0, stream,
                       static_cast<const u32x4*>(x), static_cast<const u32x4*>(r), scale, shift,
                       static_cast<u32x4*>(y), static_cast<u32x4*>(sum), nvec, cvec);
  } else {
    hipLaunchKernelGGL((bn_act_kernel<kAdd, kWriteSum, kAct, false>), dim3(blocks), dim3(256), 0, stream,
                       static_cast<const u32x4*>(x), static_cast<const u32x4*>(r), scale, shift,
                       static_cast<u32x4*>(y), static_cast<u32x4*>(sum), nvec, cvec);
  }
}

template <int kAct>
int dispatch(const void* x, const void* r, const float* scale, const float* shift, void* y, void* sum,
             unsigned nvec, unsigned cvec, bool post, hipStream_t s) {
  if (!r) launch<0, false, kAct>(x, r, scale, shift, y, sum, nvec, cvec, s);
  else if (post) launch<2, false, kAct>(x, r, scale, shift, y, sum, nvec, cvec, s);
  else if (!sum) launch<1, false, kAct>(x, r, scale, shift, y, sum, nvec, cvec, s);
  else launch<1, true, kAct>(x, r, scale, shift, y, sum, nvec, cvec, s);
  return hipGetLastError() == hipSuccess ? 0 : -2;
}

}  // namespace

extern "C" {

// x, r, y, sum: bf16 NHWC tensors of `numel` elements with `channels` innermost.
// r/sum may be null (no residual / do not materialise the sum). act: 0 none, 1 relu,
// 2 relu6. Requirements (checked): channels % 8 == 0, 16-byte aligned pointers,
// numel / 8 < 2^31. Returns 0 on success, -1 on bad arguments, -2 on launch failure.
static int bn_act_impl(const void* x, const void* r, const float* scale, const float* shift, void* y, void* sum,
                       int64_t numel, int channels, int act, bool post, void* stream) {
  if (!x || !y || !scale || !shift || channels <= 0 || channels % 8 || numel <= 0 || numel % channels) return -1;
  if (numel / 8 >= (int64_t)1 << 31) return -1;
  auto misaligned = [](const void* p) { return p && (reinterpret_cast<uintptr_t>(p) & 15u); };
  if (misaligned(x) || misaligned(r) || misaligned(y) || misaligned(sum) || misaligned(scale) || misaligned(shift))
    return -1;
  if (sum && (!r || post)) return -1;
  if (post && !r) return -1;
  const unsigned nvec = (unsigned)(numel / 8), cvec = (unsigned)(channels / 8);
  hipStream_t s = static_cast<hipStream_t>(stream);
  switch (act) {
    case 0: return dispatch<0>(x, r, scale, shift, y, sum, nvec, cvec, post, s);
    case 1: return dispatch<1>(x, r, scale, shift, y, sum, nvec, cvec, post, s);
    case 2: return dispatch<2>(x, r, scale, shift, y, sum, nvec, cvec, post, s);
    default: return -1;
  }
}

// Caps the elementwise grid at `blocks` (0 = default sizing).
void vgpu_bn_act_set_block_cap(int blocks) { g_block_cap = blocks < 0 ? 0 : blocks; }

int vgpu_bn_act_bf16(const void* x, const void* r, const float* scale, const float* shift, void* y, void* sum,
                     int64_t numel, int channels, int act, void* stream) {
  return bn_act_impl(x, r, scale, shift, y, sum, numel, channels, act, false, stream);
}

// y = act(x * scale[c] + shift[c] + r): the residual joins after the affine.
int vgpu_bn_act_post_bf16(const void* x, const void* r, const float* scale, const float* shift, void* y,
                          int64_t numel, int channels, int act, void* stream) {
  return bn_act_impl(x, r, scale, shift, y, nullptr, numel, channels, act, true, stream);
}

}  // extern "C"
