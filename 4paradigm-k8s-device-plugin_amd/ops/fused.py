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
        L.vgpu_bn_act_post_bf16.argtypes = [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p,
                                            C.c_int64, C.c_int, C.c_int, C.c_void_p]
        L.vgpu_bn_act_post_bf16.restype = C.c_int
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
