"""Fused inference ops for the benchmark models, backed by the gfx950 kernels in
``libvgpu_ops.so``: BN(eval)+activation (+ residual add) in one pass
(``native/src/kernels/fused_bn_act.hip``), and MFMA convolutions over channels-last
activations with those epilogues applied to the accumulator tile
(``native/src/kernels/conv_nhwc_mfma.hip``).

``bn_act`` / ``conv_nhwc`` are the ops; ``fuse_resnet_v2`` rewrites a
``models.aibench.ResNetV2`` for inference so that every "BN + ReLU" and every "shortcut
add + next BN + ReLU" is fused into the conv that produces its input, or else one pass
over the activation instead of 3-5 eager kernels. ``impl="torch"`` runs the same
restructured graph with plain PyTorch ops (used on CPU and as the numerics reference);
``impl="hip"`` requires the native library and a CUDA (ROCm) device and fails loudly
otherwise.
"""
import ctypes as C
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..shim.native import lib_path

OPS = os.environ.get("VGPU_OPS_LIB", "libvgpu_ops.so")  # override: A/B builds of the ops library
ACT = {"none": 0, "relu": 1, "relu6": 2}
_lib = None


def _ops():
    global _lib
    if _lib is None:
        L = C.CDLL(lib_path(OPS))
        L.vgpu_bn_act_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_int64, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_bn_act_bf16.restype = C.c_int
        L.vgpu_bn_act_post_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_int64, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_bn_act_post_bf16.restype = C.c_int
        L.vgpu_conv1x1_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                        C.c_void_p, C.c_int64, C.c_int, C.c_int, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_conv1x1_bf16.restype = C.c_int
        L.vgpu_conv_nhwc_bf16.argtypes = [C.c_void_p] * 9 + [C.c_int] * 12 + [C.c_void_p]
        L.vgpu_conv_nhwc_bf16.restype = C.c_int
        L.vgpu_conv_dual_bf16.argtypes = [C.c_void_p] * 7 + [C.c_int] * 12 + [C.c_void_p]
        L.vgpu_conv_dual_bf16.restype = C.c_int
        L.vgpu_stem_bf16.argtypes = [C.c_void_p] * 5 + [C.c_int] * 3 + [C.c_void_p]
        L.vgpu_stem_bf16.restype = C.c_int
        L.vgpu_lstm_seq_bf16.argtypes = [C.c_void_p] * 6 + [C.c_int] * 3 + [C.c_void_p]
        L.vgpu_lstm_seq_bf16.restype = C.c_int
        L.vgpu_lstm_seq_train_bf16.argtypes = [C.c_void_p] * 9 + [C.c_int] * 3 + [C.c_void_p]
        L.vgpu_lstm_seq_train_bf16.restype = C.c_int
        L.vgpu_lstm_seq_bwd_bf16.argtypes = [C.c_void_p] * 9 + [C.c_int] * 3 + [C.c_void_p]
        L.vgpu_lstm_seq_bwd_bf16.restype = C.c_int
        L.vgpu_stem_set_block_cap.argtypes = [C.c_int]
        L.vgpu_bn_act_set_block_cap.argtypes = [C.c_int]
        # Inside a CU-masked vGPU every kernel's grid is capped to one dispatch round on
        # the slice (see grid_cap): persistent stem 2 blocks/CU, elementwise 8 blocks/CU.
        slice_cus = grid_cap(128) // 2
        L.vgpu_stem_set_block_cap(slice_cus * 2)
        L.vgpu_bn_act_set_block_cap(slice_cus * 8)
        _lib = L
    return _lib


def bn_scale_shift(bn):
    """Eval-mode BatchNorm as y = x * scale + shift (fp32 per-channel vectors)."""
    inv = torch.rsqrt(bn.running_var.float() + bn.eps)
    w = bn.weight.float() if bn.weight is not None else torch.ones_like(inv)
    b = bn.bias.float() if bn.bias is not None else torch.zeros_like(inv)
    scale = w * inv
    shift = b - bn.running_mean.float() * scale
    return scale.contiguous(), shift.contiguous()


def _act_torch(y, act):
    if act == "relu":
        return F.relu(y)
    if act == "relu6":
        return F.relu6(y)
    return y


def bn_act_reference(x, scale, shift, residual=None, act="relu", post=False):
    """fp32 reference of the fused op: returns (y, sum or None). ``post``: the residual
    is added after the affine (y = act(x*s + t + r))."""
    shape = [1] * x.dim()
    shape[1] = -1
    if post:
        y = _act_torch(x.float() * scale.view(shape) + shift.view(shape) + residual.float(), act)
        return y, None
    s = x.float() + residual.float() if residual is not None else x.float()
    y = _act_torch(s * scale.view(shape) + shift.view(shape), act)
    return y, (s if residual is not None else None)


def bn_act(x, scale, shift, residual=None, act="relu", write_sum=False, post=False):
    """HIP fused op on bf16 channels-last tensors. Returns y (and the sum if write_sum).
    ``post=True`` adds the residual after the affine: y = act(x*s + t + r)."""
    if x.dtype != torch.bfloat16 or not x.is_cuda:
        raise TypeError("bn_act needs a bf16 CUDA tensor")
    if x.dim() == 4 and not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("bn_act needs channels_last input")
    C_ = x.shape[1]
    y = torch.empty_like(x, memory_format=torch.channels_last if x.dim() == 4 else torch.contiguous_format)
    s = torch.empty_like(y) if (write_sum and residual is not None) else None
    if residual is not None:
        if residual.shape != x.shape or residual.dtype != x.dtype or residual.stride() != x.stride():
            raise ValueError("residual must match x in shape, dtype and layout")
    _same_device(x, scale, shift, residual)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    if post:
        if residual is None or write_sum:
            raise ValueError("post-affine residual needs a residual and no sum output")
        rc = _ops().vgpu_bn_act_post_bf16(C.c_void_p(x.data_ptr()), C.c_void_p(residual.data_ptr()),
                                          C.c_void_p(scale.data_ptr()), C.c_void_p(shift.data_ptr()),
                                          C.c_void_p(y.data_ptr()), x.numel(), C_, ACT[act], C.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"vgpu_bn_act_post_bf16 failed ({rc}) for shape {tuple(x.shape)}")
        return y
    rc = _ops().vgpu_bn_act_bf16(C.c_void_p(x.data_ptr()),
                                 C.c_void_p(residual.data_ptr()) if residual is not None else None,
                                 C.c_void_p(scale.data_ptr()), C.c_void_p(shift.data_ptr()),
                                 C.c_void_p(y.data_ptr()), C.c_void_p(s.data_ptr()) if s is not None else None,
                                 x.numel(), C_, ACT[act], C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_bn_act_bf16 failed ({rc}) for shape {tuple(x.shape)}")
    return (y, s) if write_sum else y


def _ptr(t):
    return C.c_void_p(t.data_ptr()) if t is not None else None


def _same_device(x, *tensors):
    """Every tensor handed to a kernel must live on x's GPU: a host (or other-device)
    pointer would be dereferenced by the kernel and fault the GPU."""
    for t in tensors:
        if t is not None and t.device != x.device:
            raise ValueError(f"tensor on {t.device} passed to a kernel running on {x.device}")


def conv1x1_reference(x, w2d, scale=None, shift=None, residual=None, act="relu"):
    """fp32 reference of the fused 1x1 conv: returns (y, sum or None) as NCHW views of
    channels-last data. y = act((x . w^T [+ residual]) * scale + shift) per pixel; the
    sum is x . w^T + residual."""
    N, K, H, W = x.shape
    acc = x.permute(0, 2, 3, 1).reshape(-1, K).float() @ w2d.float().t()
    s = None
    if residual is not None:
        acc = acc + residual.permute(0, 2, 3, 1).reshape(acc.shape).float()
        s = acc
    y = acc if scale is None else _act_torch(acc * scale.float() + shift.float(), act)

    def nchw(t):
        return t.reshape(N, H, W, -1).permute(0, 3, 1, 2)

    return nchw(y), (nchw(s) if s is not None else None)


def conv1x1(x, w2d, scale=None, shift=None, residual=None, act="relu", write_sum=False):
    """HIP MFMA 1x1 convolution (``conv_nhwc_mfma.hip``) with the epilogue fused:
    y = act((x . w^T [+ residual]) * scale + shift), bf16 channels-last in and out,
    fp32 accumulation. ``w2d`` is the [Cout, Cin] weight. With ``write_sum`` also
    returns x . w^T + residual (the next block's identity shortcut)."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4:
        raise TypeError("conv1x1 needs a 4-D bf16 CUDA tensor")
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv1x1 needs channels_last input")
    N, K, H, W = x.shape
    cout = w2d.shape[0]
    if tuple(w2d.shape) != (cout, K) or w2d.dtype != torch.bfloat16 or not w2d.is_contiguous():
        raise ValueError(f"weight must be a contiguous bf16 [{cout}, {K}] matrix")
    if K % 64 or cout % 64:
        raise ValueError(f"conv1x1 needs Cin and Cout multiples of 64 (got {K}, {cout})")
    if (scale is None) != (shift is None) or (residual is not None and scale is None):
        raise ValueError("residual epilogue needs scale and shift")
    for v in (scale, shift):
        if v is not None and (v.dtype != torch.float32 or v.numel() != cout or not v.is_contiguous()):
            raise ValueError("scale/shift must be contiguous fp32 vectors of Cout")
    y = torch.empty((N, cout, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    if residual is not None and (residual.shape != y.shape or residual.dtype != y.dtype or residual.stride() != y.stride()):
        raise ValueError("residual must match the output in shape, dtype and layout")
    if write_sum and residual is None:
        raise ValueError("write_sum needs a residual")
    s = torch.empty_like(y) if write_sum else None
    epi = 0 if scale is None else 1 if residual is None else 3 if write_sum else 2
    _same_device(x, w2d, scale, shift, residual)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    rc = _ops().vgpu_conv1x1_bf16(_ptr(x), _ptr(w2d), _ptr(scale), _ptr(shift), _ptr(residual), _ptr(y), _ptr(s),
                                  N * H * W, cout, K, epi, ACT[act], C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_conv1x1_bf16 failed ({rc}) for x {tuple(x.shape)} w {tuple(w2d.shape)}")
    return (y, s) if write_sum else y


def conv_weight_2d(w):
    """[Cout, KH*KW*Cin] view of a conv weight in (kh, kw, c) order, the K order of the
    implicit GEMM (a view when the weight is channels_last, else a copy)."""
    return w.permute(0, 2, 3, 1).reshape(w.shape[0], -1).contiguous()


def conv_reference(x, w, stride=1, padding=0, scale=None, shift=None, residual=None, act="relu", post=False,
                   prologue=None):
    """fp32 reference of :func:`conv_nhwc`: returns (y, sum or None). ``prologue``:
    (scale, shift) applied as relu(x * scale + shift) to the input, rounded to x's dtype
    as the kernel stages it."""
    shape = [1, -1, 1, 1]
    if prologue is not None:
        ps, pt = prologue
        x = F.relu(x.float() * ps.float().view(shape) + pt.float().view(shape)).to(x.dtype)
    acc = F.conv2d(x.float(), w.float(), stride=stride, padding=padding)
    s = None
    if residual is not None and not post:
        acc = acc + residual.float()
        s = acc
    if scale is None:
        return acc, s
    y = acc * scale.float().view(shape) + shift.float().view(shape)
    if post:
        y = y + residual.float()
    return _act_torch(y, act), s


def grid_cap(cout, device=None):
    """Block cap for :func:`conv_nhwc` inside a CU-masked vGPU: the slice's capacity
    (CUs x blocks per CU of the chosen tile), so a launch is placed in one round
    (profiles/r1z: multi-round grids of masked tenants stall each other's dispatch).
    0 (no cap) outside a spatially limited vGPU. Reads the vGPU contract env
    (VGPU_DEVICE_CU_LIMIT, VGPU_CU_MODE) the container was started with."""
    try:
        pct = int(os.environ.get("VGPU_DEVICE_CU_LIMIT", os.environ.get("VGPU_DEVICE_CU_LIMIT_0", "0")))
    except ValueError:
        return 0
    if not 0 < pct < 100 or os.environ.get("VGPU_CU_MODE", "spatial") not in ("spatial", "both"):
        return 0
    cus = torch.cuda.get_device_properties(device if device is not None else torch.cuda.current_device()).multi_processor_count
    slice_cus = max(8, cus * pct // 100 // 8 * 8)  # masks are XCD-balanced (8 XCDs)
    return slice_cus * (2 if cout % 128 == 0 else 3)


def conv_nhwc(x, w, stride=1, padding=0, scale=None, shift=None, residual=None, act="relu", write_sum=False,
              post=False, w2d=None, prologue=None, max_blocks=None):
    """HIP MFMA convolution (``conv_nhwc_mfma.hip``: implicit GEMM over channels-last
    activations) with the epilogue fused: y = act((conv(x, w) [+ residual]) * scale +
    shift), or with ``post`` act(conv * scale + shift + residual), or without scale/shift
    conv (+ residual). ``w`` is the 4-D conv weight (``w2d``: its cached
    :func:`conv_weight_2d`). ``prologue`` = (scale, shift): the input is read as
    relu(x * scale + shift) (1x1 stride-1 convs with a BN + ReLU epilogue). Cin and Cout
    must be multiples of 64; padding symmetric and smaller than the kernel."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4:
        raise TypeError("conv_nhwc needs a 4-D bf16 CUDA tensor")
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("conv_nhwc needs channels_last input")
    N, Cin, H, W = x.shape
    cout, cin_w, kh, kw = w.shape
    if cin_w != Cin or w.dtype != torch.bfloat16:
        raise ValueError(f"weight {tuple(w.shape)} does not match input channels {Cin}")
    if Cin % 64 or cout % 64:
        raise ValueError(f"conv_nhwc needs Cin and Cout multiples of 64 (got {Cin}, {cout})")
    if not (0 <= padding < min(kh, kw)) or stride < 1:
        raise ValueError("unsupported stride/padding")
    w2d = conv_weight_2d(w) if w2d is None else w2d
    if tuple(w2d.shape) != (cout, kh * kw * Cin) or not w2d.is_contiguous():
        raise ValueError("w2d must be the contiguous [Cout, KH*KW*Cin] weight")
    if (scale is None) != (shift is None) or (residual is not None and scale is None and (post or write_sum)):
        raise ValueError("post-BN residual and sum output need scale and shift")
    for v in (scale, shift):
        if v is not None and (v.dtype != torch.float32 or v.numel() != cout or not v.is_contiguous()):
            raise ValueError("scale/shift must be contiguous fp32 vectors of Cout")
    ps = pt = None
    if prologue is not None:
        ps, pt = prologue
        if (kh, kw, stride, padding) != (1, 1, 1, 0) or scale is None or residual is not None or act != "relu":
            raise ValueError("the input prologue is for 1x1 stride-1 convs with a BN + ReLU epilogue")
        for v in (ps, pt):
            if v.dtype != torch.float32 or v.numel() != Cin or not v.is_contiguous():
                raise ValueError("prologue scale/shift must be contiguous fp32 vectors of Cin")
    oh, ow = (H + 2 * padding - kh) // stride + 1, (W + 2 * padding - kw) // stride + 1
    y = torch.empty((N, cout, oh, ow), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    if residual is not None and (residual.shape != y.shape or residual.dtype != y.dtype or residual.stride() != y.stride()):
        raise ValueError("residual must match the output in shape, dtype and layout")
    if write_sum and (residual is None or post):
        raise ValueError("write_sum needs a pre-BN residual")
    s = torch.empty_like(y) if write_sum else None
    if scale is None:
        epi = 0 if residual is None else 5
    elif residual is None:
        epi = 1
    else:
        epi = 4 if post else 3 if write_sum else 2
    _same_device(x, w2d, scale, shift, residual, ps, pt)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    if max_blocks is None:
        max_blocks = grid_cap(cout, x.device)
    rc = _ops().vgpu_conv_nhwc_bf16(_ptr(x), _ptr(w2d), _ptr(scale), _ptr(shift), _ptr(residual), _ptr(y), _ptr(s),
                                    _ptr(ps), _ptr(pt), N, H, W, Cin, cout, kh, kw, stride, padding, epi, ACT[act],
                                    int(max_blocks), C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_conv_nhwc_bf16 failed ({rc}) for x {tuple(x.shape)} w {tuple(w.shape)}")
    return (y, s) if write_sum else y


def conv_dual_reference(x, w1, x2, w2, stride2=1, scale=None, shift=None, act="relu"):
    """fp32 reference of :func:`conv_dual`: returns (y, acc)."""
    acc = F.conv2d(x.float(), w1.float()) + F.conv2d(x2.float(), w2.float(), stride=stride2)
    if scale is None:
        return acc, acc
    shape = [1, -1, 1, 1]
    return _act_torch(acc * scale.float().view(shape) + shift.float().view(shape), act), acc


def conv_dual_weight(w1, w2):
    """[Cout, C + C2] weight of :func:`conv_dual` from two 1x1 conv weights."""
    return torch.cat([conv_weight_2d(w1), conv_weight_2d(w2)], dim=1).contiguous()


def conv_dual(x, x2, wcat, stride2=1, scale=None, shift=None, act="relu", write_sum=False, max_blocks=None):
    """One MFMA GEMM for a projection block's conv3 and its shortcut conv
    (``conv_nhwc_mfma.hip``, dual source): acc = conv1x1(x, w1) + conv1x1(x2, w2,
    stride2), ``wcat`` = :func:`conv_dual_weight` (w1 | w2 along K). Returns acc, or
    act(acc * scale + shift) (and acc too with ``write_sum``). The shortcut output is
    never written to HBM and read back as a residual."""
    for t in (x, x2):
        if t.dtype != torch.bfloat16 or not t.is_cuda or t.dim() != 4 or \
                not t.is_contiguous(memory_format=torch.channels_last):
            raise TypeError("conv_dual needs 4-D bf16 channels_last CUDA tensors")
    N, Cin, H, W = x.shape
    N2, C2, H2, W2 = x2.shape
    cout = wcat.shape[0]
    if N2 != N or (H2 - 1) // stride2 + 1 != H or (W2 - 1) // stride2 + 1 != W:
        raise ValueError(f"x2 {tuple(x2.shape)} with stride {stride2} does not map onto x {tuple(x.shape)}")
    if tuple(wcat.shape) != (cout, Cin + C2) or wcat.dtype != torch.bfloat16 or not wcat.is_contiguous():
        raise ValueError("wcat must be the contiguous bf16 [Cout, C + C2] weight")
    if Cin % 64 or C2 % 64 or cout % 64:
        raise ValueError("conv_dual needs channel counts that are multiples of 64")
    if (scale is None) != (shift is None) or (write_sum and scale is None):
        raise ValueError("write_sum needs scale and shift")
    for v in (scale, shift):
        if v is not None and (v.dtype != torch.float32 or v.numel() != cout or not v.is_contiguous()):
            raise ValueError("scale/shift must be contiguous fp32 vectors of Cout")
    y = torch.empty((N, cout, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    s = torch.empty_like(y) if write_sum else None
    epi = 0 if scale is None else 6 if write_sum else 1
    _same_device(x, x2, wcat, scale, shift)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    if max_blocks is None:
        max_blocks = grid_cap(cout, x.device)
    rc = _ops().vgpu_conv_dual_bf16(_ptr(x), _ptr(x2), _ptr(wcat), _ptr(scale), _ptr(shift), _ptr(y), _ptr(s), N, H,
                                    W, Cin, C2, H2, W2, stride2, cout, epi, ACT[act], int(max_blocks),
                                    C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_conv_dual_bf16 failed ({rc}) for x {tuple(x.shape)} x2 {tuple(x2.shape)}")
    return (y, s) if write_sum else y


def is_resnet_stem(conv, pool):
    """conv7x7/2 (3 -> 64, pad 3, no bias) followed by maxpool3x3/2 pad 1: the shape
    ``stem_mfma.hip`` fuses."""
    return (isinstance(conv, nn.Conv2d) and conv.in_channels == 3 and conv.out_channels == 64
            and conv.kernel_size == (7, 7) and conv.stride == (2, 2) and conv.padding == (3, 3)
            and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and isinstance(pool, nn.MaxPool2d) and pool.kernel_size in (3, (3, 3)) and pool.stride in (2, (2, 2))
            and pool.padding in (1, (1, 1)) and pool.dilation in (1, (1, 1)) and not pool.ceil_mode)


def stem_weight(w):
    """[64, 192] matrix of a [64, 3, 7, 7] stem weight in the kernel's K order: 24 groups
    of 8 = (kh, c) pairs x kw padded 7 -> 8, groups 21..23 zero."""
    cout = w.shape[0]
    m = torch.zeros(cout, 24, 8, dtype=w.dtype, device=w.device)
    m[:, :21, :7] = w.permute(0, 2, 1, 3).reshape(cout, 21, 7)
    return m.reshape(cout, 192).contiguous()


def stem_reference(x, w, scale, shift):
    """fp32 reference: relu(bn(maxpool3x3/2(conv7x7/2(x))))."""
    y = F.max_pool2d(F.conv2d(x.float(), w.float(), stride=2, padding=3), 3, 2, 1)
    return F.relu(y * scale.float().view(1, -1, 1, 1) + shift.float().view(1, -1, 1, 1))


def stem_pool_bn_act(x, w192, scale, shift):
    """HIP fused ResNet stem (``stem_mfma.hip``): conv7x7/2 + maxpool3x3/2 + BN + ReLU in
    one kernel on bf16 channels-last input; ``w192`` from :func:`stem_weight`."""
    if x.dtype != torch.bfloat16 or not x.is_cuda or x.dim() != 4 or x.shape[1] != 3:
        raise TypeError("stem needs a [N, 3, H, W] bf16 CUDA tensor")
    if not x.is_contiguous(memory_format=torch.channels_last):
        raise ValueError("stem needs channels_last input")
    if tuple(w192.shape) != (64, 192) or w192.dtype != torch.bfloat16 or not w192.is_contiguous():
        raise ValueError("w192 must be the contiguous [64, 192] bf16 stem matrix")
    for v in (scale, shift):
        if v.dtype != torch.float32 or v.numel() != 64 or not v.is_contiguous():
            raise ValueError("scale/shift must be contiguous fp32 vectors of 64")
    N, _, H, W = x.shape
    ch, cw = (H - 1) // 2 + 1, (W - 1) // 2 + 1
    ph, pw = (ch - 1) // 2 + 1, (cw - 1) // 2 + 1
    y = torch.empty((N, 64, ph, pw), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
    _same_device(x, w192, scale, shift)
    stream = torch.cuda.current_stream(x.device).cuda_stream
    rc = _ops().vgpu_stem_bf16(_ptr(x), _ptr(w192), _ptr(scale), _ptr(shift), _ptr(y), N, H, W, C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_stem_bf16 failed ({rc}) for x {tuple(x.shape)}")
    return y


def is_mfma_conv(conv, allow_bias=False):
    """A dense convolution the MFMA kernel tiles: channels multiples of 64, square stride
    and symmetric padding smaller than the kernel, no dilation, no bias (unless the
    caller folds it into the epilogue shift)."""
    if not isinstance(conv, nn.Conv2d) or conv.groups != 1 or conv.dilation != (1, 1):
        return False
    if conv.bias is not None and not allow_bias:
        return False
    if conv.in_channels % 64 or conv.out_channels % 64 or not isinstance(conv.padding, tuple):
        return False
    (sh, sw), (ph, pw), (kh, kw) = conv.stride, conv.padding, conv.kernel_size
    return sh == sw and ph == pw and ph < min(kh, kw)


def is_pointwise(conv):
    """A bias-free 1x1/stride-1 convolution whose channels the MFMA kernel tiles."""
    return (isinstance(conv, nn.Conv2d) and conv.kernel_size == (1, 1) and conv.stride == (1, 1)
            and conv.padding == (0, 0) and conv.dilation == (1, 1) and conv.groups == 1 and conv.bias is None
            and conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0)


def _time_us(fn, reps=5):
    fn()
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    e.synchronize()
    return s.elapsed_time(e) * 1000.0 / reps


class FusedBNAct(nn.Module):
    """Frozen BN + activation (+ optional residual add)."""

    def __init__(self, bn, act="relu", impl="hip", post=False):
        super().__init__()
        scale, shift = bn_scale_shift(bn)
        self.register_buffer("scale", scale)
        self.register_buffer("shift", shift)
        self.act, self.impl, self.post = act, impl, post

    def forward(self, x, residual=None, write_sum=False):
        if self.impl == "hip":
            return bn_act(x, self.scale, self.shift, residual, self.act, write_sum, post=self.post and residual is not None)
        y, s = bn_act_reference(x, self.scale, self.shift, residual, self.act, post=self.post and residual is not None)
        y = y.to(x.dtype).contiguous(memory_format=torch.channels_last) if x.dim() == 4 else y.to(x.dtype)
        if write_sum:
            return y, s.to(x.dtype).contiguous(memory_format=torch.channels_last)
        return y


class FusedResNetV2(nn.Module):
    """Inference form of ``models.aibench.ResNetV2`` with fused epilogues.

    Per block (pre-activation bottleneck): pre = act(bn1(x)) arrives precomputed;
    y = conv1(pre) -> [bn2+relu] -> conv2 -> [bn3+relu] -> conv3; the block boundary
    computes x' = y + shortcut and pre' = act(bn1'(x')) in one kernel (bn1' = next
    block's bn1, or the final post_bn).

    Every conv can also take its epilogue inside the conv: the MFMA kernel of
    :func:`conv_nhwc` computes conv1 + bn2 + ReLU, conv2 (3x3, implicit GEMM) + bn3 +
    ReLU, the strided shortcut, and conv3 + shortcut + next BN + ReLU (+ the sum), so no
    conv output round-trips through HBM before its elementwise pass. ``mfma_conv``:
    "on", "off" or "auto" (default, env ``VGPU_MFMA_CONV``): per layer, the first forward
    times the fused kernel against library conv + separate epilogue and keeps the faster
    (like MIOpen find mode).
    """

    def __init__(self, model, impl="hip", mfma_conv=None):
        super().__init__()
        self.impl = impl
        self.mfma_mode = mfma_conv or os.environ.get("VGPU_MFMA_CONV", os.environ.get("VGPU_CONV1X1", "auto"))
        if self.mfma_mode not in ("on", "off", "auto"):
            raise ValueError(f"mfma_conv mode must be on, off or auto (got {self.mfma_mode!r})")
        self.plan = {}      # (block, conv, input shape) -> fused kernel chosen
        self._wcache = {}   # conv id -> (weight data_ptr, dtype, [Cout, KH*KW*Cin] matrix)
        self.stem, self.pool, self.fc = model.stem, model.pool, model.fc
        blocks = list(model.blocks)
        self.convs = nn.ModuleList()
        self.shortcuts = nn.ModuleList()
        self.mid = nn.ModuleList()
        for b in blocks:
            self.convs.append(nn.ModuleList([b.conv1, b.conv2, b.conv3]))
            self.shortcuts.append(b.shortcut if b.shortcut is not None else nn.Identity())
            self.mid.append(nn.ModuleList([FusedBNAct(b.bn2, "relu", impl), FusedBNAct(b.bn3, "relu", impl)]))
        self.has_sc = [b.shortcut is not None for b in blocks]
        self.entry = FusedBNAct(blocks[0].bn1, "relu", impl)
        self.boundary = nn.ModuleList([FusedBNAct(blocks[i + 1].bn1, "relu", impl) for i in range(len(blocks) - 1)] +
                                      [FusedBNAct(model.post_bn, "relu", impl)])
        self.eligible = [(is_mfma_conv(b.conv1), is_mfma_conv(b.conv2), is_mfma_conv(b.conv3),
                          b.shortcut is not None and is_mfma_conv(b.shortcut)) for b in blocks]
        # Fused stem (conv + pool + first BN/ReLU) needs block 0 to project its shortcut
        # from `pre`, since the pooled map itself is never materialised.
        self.stem_fusable = is_resnet_stem(model.stem, model.pool) and self.has_sc[0]
        # Block j's conv1 reads x and applies bn1_j + ReLU itself (the previous conv3 then
        # writes only x) when pre_j has no other reader (identity shortcut) and both convs
        # run on the MFMA kernel: one full activation write and read fewer per block. Not
        # timed in "auto". The prologue is applied to conv1's A fragments as they leave LDS
        # (profiles/r1at: 23700 -> 24353 img/s over a rule that kept compute-bound conv1s
        # plain, which the earlier register-staged prologue had doubled; r1as).
        # VGPU_PROLOGUE=off disables it (measurement).
        on = self.mfma_mode == "on" or (self.mfma_mode == "auto" and impl == "hip")
        pmode = os.environ.get("VGPU_PROLOGUE", "on")
        self.prologue = [on and pmode != "off" and j > 0 and not self.has_sc[j] and is_pointwise(blocks[j].conv1)
                         and self.eligible[j - 1][2] for j in range(len(blocks))]
        # Projection blocks: conv3 and the 1x1 shortcut conv run as one GEMM over
        # [y | pre strided] (conv_dual), so the shortcut output never round-trips through
        # HBM as conv3's residual. Not timed in "auto" either: it removes a full
        # activation write and read and the shortcut's launch.
        self.dual = [on and b.shortcut is not None and self.eligible[j][2] and self.eligible[j][3]
                     and is_pointwise(b.conv3) and b.shortcut.kernel_size == (1, 1) and b.shortcut.padding == (0, 0)
                     and b.shortcut.stride[0] == b.shortcut.stride[1] for j, b in enumerate(blocks)]

    def _w2d(self, conv):
        w = conv.weight
        hit = self._wcache.get(id(conv))
        if hit is None or hit[0] != w.data_ptr() or hit[1] != w.dtype:
            hit = (w.data_ptr(), w.dtype, conv_weight_2d(w.detach()))
            self._wcache[id(conv)] = hit
        return hit[2]

    def _conv(self, x, conv, bn=None, residual=None, write_sum=False, prologue=None):
        """conv with bn's epilogue (and optionally the input's BN + ReLU as a prologue)
        fused: the HIP MFMA kernel, or its fp32 torch reference for impl="torch"."""
        st, pad = conv.stride[0], conv.padding[0]
        sc, sh, act = (bn.scale, bn.shift, bn.act) if bn is not None else (None, None, "none")
        pro = (prologue.scale, prologue.shift) if prologue is not None else None
        if self.impl == "hip":
            return conv_nhwc(x, conv.weight, st, pad, sc, sh, residual, act, write_sum, w2d=self._w2d(conv),
                             prologue=pro)
        y, s = conv_reference(x, conv.weight, st, pad, sc, sh, residual, act, prologue=pro)
        y = y.to(x.dtype).contiguous(memory_format=torch.channels_last)
        return (y, s.to(x.dtype).contiguous(memory_format=torch.channels_last)) if write_sum else y

    def _dual(self, i, y, pre, bn=None, write_sum=False):
        """Block i's conv3(y) + shortcut(pre) as one GEMM, with bn's epilogue (and the
        pre-BN sum with write_sum)."""
        c3, scv = self.convs[i][2], self.shortcuts[i]
        st = scv.stride[0]
        sc, sh, act = (bn.scale, bn.shift, bn.act) if bn is not None else (None, None, "none")
        if self.impl == "hip":
            key = ("dual", i)
            hit = self._wcache.get(key)
            tag = (c3.weight.data_ptr(), scv.weight.data_ptr(), c3.weight.dtype)
            if hit is None or hit[0] != tag:
                hit = self._wcache[key] = (tag, conv_dual_weight(c3.weight.detach(), scv.weight.detach()))
            return conv_dual(y, pre, hit[1], st, sc, sh, act, write_sum)
        out, acc = conv_dual_reference(y, c3.weight, pre, scv.weight, st, sc, sh, act)
        out = out.to(y.dtype).contiguous(memory_format=torch.channels_last)
        return (out, acc.to(y.dtype).contiguous(memory_format=torch.channels_last)) if write_sum else out

    def _use(self, key, fused, unfused):
        if self.mfma_mode != "auto" or self.impl != "hip":
            return self.mfma_mode == "on"
        d = self.plan.get(key)
        if d is None:
            if torch.cuda.is_current_stream_capturing():
                return True  # no timing inside a graph capture: take the kernel
            d = self.plan[key] = _time_us(fused) <= _time_us(unfused)
        return d

    def _stem_fused(self, x):
        if self.impl == "hip":
            w = self.stem.weight
            hit = self._wcache.get("stem")
            if hit is None or hit[0] != w.data_ptr() or hit[1] != w.dtype:
                hit = self._wcache["stem"] = (w.data_ptr(), w.dtype, stem_weight(w.detach()))
            return stem_pool_bn_act(x, hit[2], self.entry.scale, self.entry.shift)
        y = stem_reference(x, self.stem.weight, self.entry.scale, self.entry.shift)
        return y.to(x.dtype).contiguous(memory_format=torch.channels_last)

    def forward(self, x):
        if self.stem_fusable and self._use(("stem", tuple(x.shape)), lambda: self._stem_fused(x),
                                           lambda: self.entry(self.pool(self.stem(x)))):
            pre, x = self._stem_fused(x), None  # block 0 projects its shortcut from pre
        else:
            x = self.pool(self.stem(x))
            pre = self.entry(x)
        n = len(self.convs)
        for i in range(n):
            c1, c2, c3 = self.convs[i]
            bn2, bn3 = self.mid[i]
            bnd, last = self.boundary[i], i + 1 == n
            e1, e2, e3, esc = self.eligible[i]
            # pre is None when the previous conv3 wrote only x: this block's conv1 then
            # applies its pre-activation BN + ReLU (bn_in) while loading x.
            bn_in = self.entry if i == 0 else self.boundary[i - 1]
            if self.dual[i]:
                sc = None  # folded into conv3 (conv_dual)
            elif not self.has_sc[i]:
                sc = x
            elif esc and self._use((i, 0, tuple(pre.shape)), lambda: self._conv(pre, self.shortcuts[i]),
                                   lambda: self.shortcuts[i](pre)):
                sc = self._conv(pre, self.shortcuts[i])
            else:
                sc = self.shortcuts[i](pre)
            if pre is None:
                y = self._conv(x, c1, bn2, prologue=bn_in)
            elif e1 and self._use((i, 1, tuple(pre.shape)), lambda: self._conv(pre, c1, bn2), lambda: bn2(c1(pre))):
                y = self._conv(pre, c1, bn2)
            else:
                y = bn2(c1(pre))
            if e2 and self._use((i, 2, tuple(y.shape)), lambda: self._conv(y, c2, bn3), lambda: bn3(c2(y))):
                y = self._conv(y, c2, bn3)
            else:
                y = bn3(c2(y))
            if self.dual[i]:
                if not last and self.prologue[i + 1]:
                    x, pre = self._dual(i, y, pre), None
                elif last:
                    pre, x = self._dual(i, y, pre, bnd), None
                else:
                    pre, x = self._dual(i, y, pre, bnd, write_sum=True)
            elif not last and self.prologue[i + 1]:
                x, pre = self._conv(y, c3, None, sc), None  # next conv1 applies bnd itself
            else:
                # x itself is only read as the next block's identity shortcut: not after the
                # last block, and not before a dual projection block (which reads pre only).
                ws = not last and not self.dual[i + 1]
                if e3 and self._use((i, 3, tuple(y.shape)), lambda: self._conv(y, c3, bnd, sc, ws),
                                    lambda: bnd(c3(y), residual=sc, write_sum=ws)):
                    out = self._conv(y, c3, bnd, sc, ws)
                else:
                    out = bnd(c3(y), residual=sc, write_sum=ws)
                pre, x = out if ws else (out, None)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(pre, 1), 1))


def fuse_resnet_v2(model, impl="hip", mfma_conv=None):
    model.eval()
    return FusedResNetV2(model, impl, mfma_conv).eval()


class ConvBiasAct(nn.Module):
    """Conv2d(+bias) + ReLU as one MFMA kernel (:func:`conv_nhwc` with scale 1 and the
    bias as shift): the VGG pattern. Falls back to library conv + ReLU for shapes the
    kernel does not tile; in "auto" mode (env ``VGPU_MFMA_CONV``) the first forward per
    input shape times both and keeps the faster."""

    def __init__(self, conv, act="relu", impl="hip", mfma_conv=None):
        super().__init__()
        self.conv, self.act, self.impl = conv, act, impl
        self.mode = mfma_conv or os.environ.get("VGPU_MFMA_CONV", os.environ.get("VGPU_CONV1X1", "auto"))
        dev = conv.weight.device
        bias = conv.bias.detach().float() if conv.bias is not None else torch.zeros(conv.out_channels, device=dev)
        self.register_buffer("shift", bias.contiguous())
        self.register_buffer("scale", torch.ones(conv.out_channels, device=dev))
        self.eligible = is_mfma_conv(conv, allow_bias=True)
        self.plan = {}
        self._w = None

    def _library(self, x):
        return _act_torch(self.conv(x), self.act)

    def _fused(self, x):
        w = self.conv.weight
        if self._w is None or self._w[0] != w.data_ptr() or self._w[1] != w.dtype:
            self._w = (w.data_ptr(), w.dtype, conv_weight_2d(w.detach()))
        return conv_nhwc(x, w, self.conv.stride[0], self.conv.padding[0], self.scale, self.shift, act=self.act,
                         w2d=self._w[2])

    def forward(self, x):
        ok = (self.eligible and self.impl == "hip" and self.mode != "off" and x.is_cuda and x.dtype == torch.bfloat16
              and x.is_contiguous(memory_format=torch.channels_last))
        if not ok:
            return self._library(x)
        if self.mode == "on":
            return self._fused(x)
        key = tuple(x.shape)
        d = self.plan.get(key)
        if d is None:
            if torch.cuda.is_current_stream_capturing():
                return self._fused(x)
            d = self.plan[key] = _time_us(lambda: self._fused(x)) <= _time_us(lambda: self._library(x))
        return self._fused(x) if d else self._library(x)


def fuse_conv_relu(model, impl="hip", mfma_conv=None):
    """In-place inference rewrite of every (Conv2d, ReLU) pair inside a Sequential into a
    :class:`ConvBiasAct` (the ReLU becomes Identity)."""
    model.eval()
    for child in model.children():
        if isinstance(child, nn.Sequential):
            mods = list(child)
            for j in range(len(mods) - 1):
                if isinstance(mods[j], nn.Conv2d) and isinstance(mods[j + 1], nn.ReLU):
                    child[j] = ConvBiasAct(mods[j], "relu", impl, mfma_conv)
                    child[j + 1] = nn.Identity()
        fuse_conv_relu(child, impl, mfma_conv)
    return model


def lstm_recurrence(gx, whh, h0=None, c0=None):
    """HIP LSTM recurrence (``lstm_mfma.hip``) over a whole sequence: ``gx`` [B, T, 128, 4]
    bf16 gate inputs (x . W_ih^T + b, gates i, f, g, o of a unit adjacent), ``whh`` the
    [512, 128] bf16 weight_hh. Returns (h_T, c_T) fp32 [B, 128]."""
    if gx.dtype != torch.bfloat16 or not gx.is_cuda or gx.dim() != 4 or gx.shape[2:] != (128, 4):
        raise TypeError("gx must be a [B, T, 128, 4] bf16 CUDA tensor")
    if not gx.is_contiguous() or tuple(whh.shape) != (512, 128) or whh.dtype != torch.bfloat16 or not whh.is_contiguous():
        raise ValueError("gx must be contiguous and whh a contiguous [512, 128] bf16 matrix")
    B, T = gx.shape[:2]
    for t in (h0, c0):
        if t is not None and (t.dtype != torch.float32 or tuple(t.shape) != (B, 128) or not t.is_contiguous()):
            raise ValueError("h0/c0 must be contiguous fp32 [B, 128]")
    hT = torch.empty(B, 128, dtype=torch.float32, device=gx.device)
    cT = torch.empty_like(hT)
    _same_device(gx, whh, h0, c0)
    stream = torch.cuda.current_stream(gx.device).cuda_stream
    rc = _ops().vgpu_lstm_seq_bf16(_ptr(gx), _ptr(whh), _ptr(h0), _ptr(c0), _ptr(hT), _ptr(cT), B, T, 128,
                                   C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_lstm_seq_bf16 failed ({rc}) for gx {tuple(gx.shape)}")
    return hT, cT


# Buffer-descriptor ranges of the LSTM kernels (lstm_mfma.hip host guards): the stash of
# the training kernel holds B*T*128*16 bytes, the inference input B*T*128*8; both must stay
# below 2^31. Larger inputs take the library LSTM instead of failing.
LSTM_TRAIN_MAX_BT = (1 << 31) // (128 * 16)
LSTM_INFER_MAX_BT = (1 << 31) // (128 * 8)


def lstm_fits(x, max_bt):
    return x.dim() == 3 and x.shape[0] * x.shape[1] < max_bt


class FusedLSTMLast(nn.Module):
    """Inference form of a single-layer, unidirectional, batch-first ``nn.LSTM`` with 128
    hidden units whose caller only needs the last hidden state (the sentiment model):
    one library GEMM for the input projection of every step (W_ih rows permuted so a
    unit's four gates are adjacent), then the whole recurrence in one HIP kernel. The
    original module stays as the library path for "off" / "auto" (``VGPU_MFMA_CONV``
    governs the in-pod kernels)."""

    def __init__(self, lstm, impl="hip", mode=None):
        super().__init__()
        if (lstm.num_layers != 1 or lstm.bidirectional or not lstm.batch_first or lstm.hidden_size != 128
                or not lstm.bias or getattr(lstm, "proj_size", 0)):
            raise ValueError("FusedLSTMLast needs a 1-layer, unidirectional, batch-first LSTM with 128 units")
        self.lstm, self.impl = lstm, impl
        self.mode = mode or os.environ.get("VGPU_MFMA_CONV", os.environ.get("VGPU_CONV1X1", "auto"))
        H, Fin = lstm.hidden_size, lstm.input_size
        w = lstm.weight_ih_l0.detach().float().view(4, H, Fin).permute(1, 0, 2).reshape(4 * H, Fin)
        b = (lstm.bias_ih_l0.detach().float() + lstm.bias_hh_l0.detach().float()).view(4, H).t().reshape(4 * H)
        self.register_buffer("w_ih_perm", w.contiguous())
        self.register_buffer("b_perm", b.contiguous())
        self.plan = {}
        self._cast = None
        self._src = None

    def _weights_version(self):
        l = self.lstm
        return tuple((p.data_ptr(), p._version) for p in (l.weight_ih_l0, l.weight_hh_l0, l.bias_ih_l0, l.bias_hh_l0))

    def _refresh(self):
        """Re-derives the permuted weights when the wrapped LSTM's parameters changed
        (load_state_dict, fine-tuning, the library path's in-place .to(dtype))."""
        v = self._weights_version()
        if v == self._src:
            return
        l, H, Fin = self.lstm, self.lstm.hidden_size, self.lstm.input_size
        with torch.no_grad():
            w = l.weight_ih_l0.detach().float().view(4, H, Fin).permute(1, 0, 2).reshape(4 * H, Fin)
            b = (l.bias_ih_l0.detach().float() + l.bias_hh_l0.detach().float()).view(4, H).t().reshape(4 * H)
            self.w_ih_perm = w.contiguous().to(self.w_ih_perm.device)
            self.b_perm = b.contiguous().to(self.b_perm.device)
        self._cast = None
        self._src = v

    def _fused(self, x):
        self._refresh()
        if self._cast is None or self._cast[0] != x.dtype:
            self._cast = (x.dtype, self.w_ih_perm.to(x.dtype).t(), self.b_perm.to(x.dtype),
                          self.lstm.weight_hh_l0.detach().to(x.dtype).contiguous())
        _, wt, b, whh = self._cast
        B, T, Fin = x.shape
        gx = torch.addmm(b, x.reshape(B * T, Fin), wt).view(B, T, 128, 4)
        hT, _ = lstm_recurrence(gx, whh)
        return hT.to(x.dtype)

    def _library(self, x):
        if next(self.lstm.parameters()).dtype != x.dtype:
            self.lstm.to(x.dtype)
        out, _ = self.lstm(x)
        return out[:, -1]

    def forward(self, x):
        ok = (self.impl == "hip" and self.mode != "off" and x.is_cuda and x.dtype == torch.bfloat16
              and lstm_fits(x, LSTM_INFER_MAX_BT))
        if not ok:
            return self._library(x)
        if self.mode == "on":
            return self._fused(x)
        key = tuple(x.shape)
        d = self.plan.get(key)
        if d is None:
            if torch.cuda.is_current_stream_capturing():
                return self._fused(x)
            d = self.plan[key] = _time_us(lambda: self._fused(x)) <= _time_us(lambda: self._library(x))
        return self._fused(x) if d else self._library(x)


def lstm_input_projection(x, w_ih, b_ih, b_hh, dtype):
    """gx [B, T, 128, 4] = x . W_ih^T + b_ih + b_hh with W_ih's rows permuted so the four
    gates (i, f, g, o) of one hidden unit are adjacent, the layout of ``lstm_mfma.hip``."""
    B, T, Fin = x.shape
    H = w_ih.shape[0] // 4
    w = w_ih.view(4, H, Fin).permute(1, 0, 2).reshape(4 * H, Fin).to(dtype)
    b = (b_ih.float() + b_hh.float()).view(4, H).t().reshape(4 * H).to(dtype)
    return torch.addmm(b, x.reshape(B * T, Fin).to(dtype), w.t()).view(B, T, H, 4)


def lstm_train_forward_reference(gx, w_hh, h0=None, c0=None):
    """Plain-PyTorch mirror of ``vgpu_lstm_seq_train_bf16`` (fp32 math, h rounded to the
    dtype of ``w_hh`` each step like the kernel's MFMA operand): returns hT, cT and the
    stash act [B, T, H, 4] (sigmoid i, sigmoid f, tanh g, sigmoid o), cs [B, T, H], hs."""
    B, T, H, _ = gx.shape
    dev = gx.device
    h = torch.zeros(B, H, device=dev) if h0 is None else h0.float()
    c = torch.zeros(B, H, device=dev) if c0 is None else c0.float()
    w = w_hh.float()
    act = torch.empty(B, T, H, 4, device=dev)
    cs = torch.empty(B, T, H, device=dev)
    hs = torch.empty(B, T, H, device=dev, dtype=w_hh.dtype)
    hq = h.to(w_hh.dtype).float()
    for t in range(T):
        z = gx[:, t].float() + (hq @ w.t()).view(B, 4, H).transpose(1, 2)
        i, f, g, o = torch.sigmoid(z[..., 0]), torch.sigmoid(z[..., 1]), torch.tanh(z[..., 2]), torch.sigmoid(z[..., 3])
        c = f * c + i * g
        h = o * torch.tanh(c)
        act[:, t] = torch.stack([i, f, g, o], -1)
        cs[:, t] = c
        hs[:, t] = h.to(w_hh.dtype)
        hq = hs[:, t].float()
    return h, c, act, cs, hs


def lstm_bwd_reference(w_hh, act, cs, dhT, c0=None, dcT=None):
    """Plain-PyTorch mirror of ``vgpu_lstm_seq_bwd_bf16``: BPTT of a loss on h_T over the
    forward's stash. Returns dz [B, T, 4H] (pre-activation gate gradients, columns
    i|f|g|o like PyTorch's weight rows, rounded to the dtype of ``w_hh`` like the kernel's
    MFMA operand), dh0, dc0."""
    B, T, H, _ = act.shape
    w = w_hh.float()
    dh = dhT.float()
    dc = torch.zeros_like(dh) if dcT is None else dcT.float()
    dz = torch.empty(B, T, 4 * H, device=act.device, dtype=w_hh.dtype)
    for t in range(T - 1, -1, -1):
        i, f, g, o = act[:, t].unbind(-1)
        tc = torch.tanh(cs[:, t])
        cp = cs[:, t - 1] if t > 0 else (torch.zeros_like(dh) if c0 is None else c0.float())
        dct = dc + dh * o * (1 - tc * tc)
        z = torch.cat([dct * g * i * (1 - i), dct * cp * f * (1 - f), dct * i * (1 - g * g), dh * tc * o * (1 - o)], 1)
        dc = dct * f
        dz[:, t] = z.to(w_hh.dtype)
        dh = dz[:, t].float() @ w
    return dz, dh, dc


def lstm_weight_grads(dz, x, hs, h0=None):
    """The library half of the backward: dW_ih = dz^T x, dW_hh = dz^T h_{t-1}, db = sum dz
    (one GEMM each over all B*T steps)."""
    B, T, G = dz.shape
    H = hs.shape[-1]
    first = torch.zeros(B, 1, H, device=hs.device, dtype=hs.dtype) if h0 is None else h0.to(hs.dtype).unsqueeze(1)
    hprev = torch.cat([first, hs[:, :-1]], 1).reshape(B * T, H)
    dzf = dz.reshape(B * T, G)
    dw_ih = dzf.t().mm(x.reshape(B * T, -1).to(dz.dtype))
    dw_hh = dzf.t().mm(hprev.to(dz.dtype))
    db = dzf.float().sum(0)
    return dw_ih, dw_hh, db


class _LSTMLastFn(torch.autograd.Function):
    """h_T of a 1-layer, 128-unit LSTM with zero initial state, forward and backward on the
    whole-sequence HIP kernels (``lstm_mfma.hip``): input projection (library GEMM) →
    stashing recurrence kernel; backward recurrence kernel → three library GEMMs for the
    weight gradients. Every piece runs on the current stream, so the training step is
    HIP-graph capturable (MIOpen's RNN backward is not)."""

    @staticmethod
    def forward(ctx, x, w_ih, w_hh, b_ih, b_hh):
        dt = torch.bfloat16
        gx = lstm_input_projection(x, w_ih, b_ih, b_hh, dt).contiguous()
        whh = w_hh.to(dt).contiguous()
        B, T = x.shape[:2]
        H = 128
        hT = torch.empty(B, H, dtype=torch.float32, device=x.device)
        act = torch.empty(B, T, H, 4, dtype=torch.float32, device=x.device)
        cs = torch.empty(B, T, H, dtype=torch.float32, device=x.device)
        hs = torch.empty(B, T, H, dtype=dt, device=x.device)
        _same_device(x, whh, gx)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        rc = _ops().vgpu_lstm_seq_train_bf16(_ptr(gx), _ptr(whh), None, None, _ptr(hT), None, _ptr(act), _ptr(cs),
                                             _ptr(hs), B, T, H, C.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"vgpu_lstm_seq_train_bf16 failed ({rc}) for x {tuple(x.shape)}")
        ctx.save_for_backward(x, w_ih, whh, act, cs, hs)
        return hT.to(x.dtype)

    @staticmethod
    def backward(ctx, dhT):
        x, w_ih, whh, act, cs, hs = ctx.saved_tensors
        B, T = x.shape[:2]
        H = 128
        whhT = whh.t().contiguous()
        dh = dhT.float().contiguous()
        dz = torch.empty(B, T, 4 * H, dtype=torch.bfloat16, device=x.device)
        stream = torch.cuda.current_stream(x.device).cuda_stream
        rc = _ops().vgpu_lstm_seq_bwd_bf16(_ptr(whhT), _ptr(act), _ptr(cs), None, _ptr(dh), None, _ptr(dz), None,
                                           None, B, T, H, C.c_void_p(stream))
        if rc != 0:
            raise RuntimeError(f"vgpu_lstm_seq_bwd_bf16 failed ({rc}) for x {tuple(x.shape)}")
        dw_ih, dw_hh, db = lstm_weight_grads(dz, x, hs)
        dx = dz.reshape(B * T, 4 * H).mm(w_ih.to(dz.dtype)).view_as(x).to(x.dtype) if ctx.needs_input_grad[0] else None
        return (dx, dw_ih.to(w_ih.dtype), dw_hh.to(w_ih.dtype), db.to(w_ih.dtype), db.to(w_ih.dtype))


class FusedLSTMTrainLast(nn.Module):
    """Training form of ``FusedLSTMLast`` (the sentiment model's LSTM, only h_T used):
    forward and backward through ``_LSTMLastFn`` on the live parameters of the wrapped
    ``nn.LSTM`` (fp32 master weights, bf16 compute; gradients land in the LSTM's
    ``.grad`` like the library path's). ``VGPU_MFMA_CONV=off`` selects the library LSTM."""

    def __init__(self, lstm, mode=None):
        super().__init__()
        if (lstm.num_layers != 1 or lstm.bidirectional or not lstm.batch_first or lstm.hidden_size != 128
                or not lstm.bias or getattr(lstm, "proj_size", 0)):
            raise ValueError("FusedLSTMTrainLast needs a 1-layer, unidirectional, batch-first LSTM with 128 units")
        self.lstm = lstm
        self.mode = mode or os.environ.get("VGPU_MFMA_CONV", os.environ.get("VGPU_CONV1X1", "auto"))

    @property
    def fused(self):
        return self.mode != "off"

    def forward(self, x):
        if not self.fused or not x.is_cuda or not lstm_fits(x, LSTM_TRAIN_MAX_BT):
            out, _ = self.lstm(x)
            return out[:, -1]
        l = self.lstm
        with torch.autocast(x.device.type, enabled=False):
            return _LSTMLastFn.apply(x.to(torch.bfloat16), l.weight_ih_l0, l.weight_hh_l0, l.bias_ih_l0, l.bias_hh_l0)


class ConvBNAct(nn.Module):
    """Conv2d followed by a frozen BN + activation in one HIP pass (optionally with a
    residual joined after the BN, MobileNet-V2 style)."""

    def __init__(self, conv, bn, act, impl="hip"):
        super().__init__()
        self.conv = conv
        self.post = FusedBNAct(bn, act, impl, post=True)

    def forward(self, x, residual=None):
        return self.post(self.conv(x), residual)


def _act_name(m):
    if isinstance(m, nn.ReLU6):
        return "relu6"
    if isinstance(m, nn.ReLU):
        return "relu"
    return None


def _fuse_seq(seq, impl):
    """Sequential(Conv2d, BatchNorm2d[, ReLU|ReLU6]) -> ConvBNAct, or None."""
    mods = list(seq)
    if len(mods) in (2, 3) and isinstance(mods[0], nn.Conv2d) and isinstance(mods[1], nn.BatchNorm2d):
        act = "none" if len(mods) == 2 else _act_name(mods[2])
        if act is not None and mods[1].num_features % 8 == 0:
            return ConvBNAct(mods[0], mods[1], act, impl)
    return None


class FusedInvertedResidual(nn.Module):
    """MobileNet-V2 block whose final projection BN also adds the shortcut."""

    def __init__(self, block, impl):
        super().__init__()
        layers = [(_fuse_seq(m, impl) or m) if isinstance(m, nn.Sequential) else m for m in block.conv]
        self.body = nn.ModuleList(layers[:-1])
        self.last = layers[-1]
        self.use_res = block.use_res and isinstance(self.last, ConvBNAct)
        self.fallback = block if not isinstance(self.last, ConvBNAct) else None

    def forward(self, x):
        if self.fallback is not None:
            return self.fallback(x)
        h = x
        for m in self.body:
            h = m(h)
        return self.last(h, x if self.use_res else None)


def fuse_conv_bn_act(model, impl="hip"):
    """In-place inference rewrite of every Conv+BN(+ReLU/ReLU6) Sequential (and MobileNet
    residual blocks) of ``model`` into fused epilogues. Channels must be multiples of 8
    (others are left as they are)."""
    from ..models.aibench import InvertedResidual
    model.eval()
    for name, child in list(model.named_children()):
        if isinstance(child, InvertedResidual):
            setattr(model, name, FusedInvertedResidual(child, impl))
        elif isinstance(child, nn.Sequential) and (fused := _fuse_seq(child, impl)) is not None:
            setattr(model, name, fused)
        else:
            fuse_conv_bn_act(child, impl)
    return model
