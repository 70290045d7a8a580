"""Fused BN(eval)+activation (+ residual add) for inference, backed by the gfx950 kernel in
``native/src/kernels/fused_bn_act.hip`` (``libvgpu_ops.so``).

``bn_act`` is the op; ``fuse_resnet_v2`` rewrites a ``models.aibench.ResNetV2`` for
inference so that every "BN + ReLU" and every "shortcut add + next BN + ReLU" is one pass
over the activation instead of 3-5 eager kernels. ``impl="torch"`` runs the same
restructured graph with plain PyTorch ops (used on CPU and as the numerics reference);
``impl="hip"`` requires the native library and a CUDA (ROCm) device and fails loudly
otherwise.
"""
import ctypes as C

import torch
import torch.nn as nn
import torch.nn.functional as F

from ..shim.native import lib_path

OPS = "libvgpu_ops.so"
ACT = {"none": 0, "relu": 1, "relu6": 2}
_lib = None


def _ops():
    global _lib
    if _lib is None:
        L = C.CDLL(lib_path(OPS))
        L.vgpu_bn_act_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                       C.c_int64, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_bn_act_bf16.restype = C.c_int
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


def bn_act_reference(x, scale, shift, residual=None, act="relu"):
    """fp32 reference of the fused op: returns (y, sum or None)."""
    s = x.float() + residual.float() if residual is not None else x.float()
    shape = [1] * x.dim()
    shape[1] = -1
    y = _act_torch(s * scale.view(shape) + shift.view(shape), act)
    return y, (s if residual is not None else None)


def bn_act(x, scale, shift, residual=None, act="relu", write_sum=False):
    """HIP fused op on bf16 channels-last tensors. Returns y (and the sum if write_sum)."""
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
    stream = torch.cuda.current_stream(x.device).cuda_stream
    rc = _ops().vgpu_bn_act_bf16(C.c_void_p(x.data_ptr()),
                                 C.c_void_p(residual.data_ptr()) if residual is not None else None,
                                 C.c_void_p(scale.data_ptr()), C.c_void_p(shift.data_ptr()),
                                 C.c_void_p(y.data_ptr()), C.c_void_p(s.data_ptr()) if s is not None else None,
                                 x.numel(), C_, ACT[act], C.c_void_p(stream))
    if rc != 0:
        raise RuntimeError(f"vgpu_bn_act_bf16 failed ({rc}) for shape {tuple(x.shape)}")
    return (y, s) if write_sum else y


class FusedBNAct(nn.Module):
    """Frozen BN + activation (+ optional residual add)."""

    def __init__(self, bn, act="relu", impl="hip"):
        super().__init__()
        scale, shift = bn_scale_shift(bn)
        self.register_buffer("scale", scale)
        self.register_buffer("shift", shift)
        self.act, self.impl = act, impl

    def forward(self, x, residual=None, write_sum=False):
        if self.impl == "hip":
            return bn_act(x, self.scale, self.shift, residual, self.act, write_sum)
        y, s = bn_act_reference(x, self.scale, self.shift, residual, self.act)
        y = y.to(x.dtype).contiguous(memory_format=torch.channels_last) if x.dim() == 4 else y.to(x.dtype)
        if write_sum:
            return y, s.to(x.dtype).contiguous(memory_format=torch.channels_last)
        return y


class FusedResNetV2(nn.Module):
    """Inference form of ``models.aibench.ResNetV2`` with fused epilogues.

    Per block (pre-activation bottleneck): pre = act(bn1(x)) arrives precomputed;
    y = conv1(pre) -> [bn2+relu] -> conv2 -> [bn3+relu] -> conv3; the block boundary
    computes x' = y + shortcut and pre' = act(bn1'(x')) in one kernel (bn1' = next
    block's bn1, or the final post_bn)."""

    def __init__(self, model, impl="hip"):
        super().__init__()
        self.impl = impl
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

    def forward(self, x):
        x = self.pool(self.stem(x))
        pre = self.entry(x)
        n = len(self.convs)
        for i in range(n):
            c1, c2, c3 = self.convs[i]
            sc = self.shortcuts[i](pre) if self.has_sc[i] else x
            y = self.mid[i][0](c1(pre))
            y = self.mid[i][1](c2(y))
            y = c3(y)
            if i + 1 < n:
                pre, x = self.boundary[i](y, residual=sc, write_sum=True)
            else:
                pre = self.boundary[i](y, residual=sc)
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(pre, 1), 1))


def fuse_resnet_v2(model, impl="hip"):
    model.eval()
    return FusedResNetV2(model, impl).eval()
