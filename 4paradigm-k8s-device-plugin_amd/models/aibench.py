"""The reference's benchmark workloads, re-implemented in PyTorch for MI355X.

The reference measured its plugin with ai-benchmark on TensorFlow 2.4.1
(``benchmarks/ai-benchmark/Dockerfile:1-13``) and published ten cases
(``README.md:57-68``): ResNet-V2-50/152, VGG-16, DeepLab and LSTM, each in
inference and training. These are the same architectures at the same batch sizes and
input shapes, random-initialised, fed synthetic data (no network for datasets or
checkpoints). Inference runs the model in bf16, channels-last; training runs bf16
autocast with fp32 master weights and an SGD-momentum step (the optimizer step is part
of every timed training step).

Architecture details that ai-benchmark's frozen graphs define but the reference repo
does not (DeepLab backbone, LSTM width) are "parity unpinned": DeepLab is DeepLab-V3+
on a MobileNet-V2 backbone (output stride 16, ASPP rates 6/12/18), the LSTM is the
sentiment model shape (1024 steps x 300 features, 1 layer, 128 hidden units, 2 classes).
"""
from dataclasses import dataclass, field

import torch
import torch.nn as nn
import torch.nn.functional as F

# ----------------------------------------------------------------------------- ResNet-V2


class PreActBottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride):
        super().__init__()
        cout = width * self.expansion
        self.bn1 = nn.BatchNorm2d(cin)
        self.conv1 = nn.Conv2d(cin, width, 1, bias=False)
        self.bn2 = nn.BatchNorm2d(width)
        self.conv2 = nn.Conv2d(width, width, 3, stride=stride, padding=1, bias=False)
        self.bn3 = nn.BatchNorm2d(width)
        self.conv3 = nn.Conv2d(width, cout, 1, bias=False)
        self.shortcut = None
        if stride != 1 or cin != cout:
            self.shortcut = nn.Conv2d(cin, cout, 1, stride=stride, bias=False)

    def forward(self, x):
        pre = F.relu(self.bn1(x))
        sc = self.shortcut(pre) if self.shortcut is not None else x
        y = self.conv1(pre)
        y = self.conv2(F.relu(self.bn2(y)))
        y = self.conv3(F.relu(self.bn3(y)))
        return y + sc


class ResNetV2(nn.Module):
    """Pre-activation ResNet (He et al. 2016, "Identity Mappings"), as in TF-slim resnet_v2."""

    def __init__(self, layers, num_classes=1000):
        super().__init__()
        self.stem = nn.Conv2d(3, 64, 7, stride=2, padding=3, bias=False)
        self.pool = nn.MaxPool2d(3, stride=2, padding=1)
        blocks, cin = [], 64
        for i, n in enumerate(layers):
            width = 64 << i
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                blocks.append(PreActBottleneck(cin, width, stride))
                cin = width * 4
        self.blocks = nn.Sequential(*blocks)
        self.post_bn = nn.BatchNorm2d(cin)
        self.fc = nn.Linear(cin, num_classes)

    def forward(self, x):
        x = self.pool(self.stem(x))
        x = self.blocks(x)
        x = F.relu(self.post_bn(x))
        return self.fc(torch.flatten(F.adaptive_avg_pool2d(x, 1), 1))


def resnet_v2_50(num_classes=1000):
    return ResNetV2([3, 4, 6, 3], num_classes)


def resnet_v2_152(num_classes=1000):
    return ResNetV2([3, 8, 36, 3], num_classes)


# ----------------------------------------------------------------------------- VGG-16


class VGG16(nn.Module):
    CFG = [64, 64, "M", 128, 128, "M", 256, 256, 256, "M", 512, 512, 512, "M", 512, 512, 512, "M"]

    def __init__(self, num_classes=1000):
        super().__init__()
        layers, cin = [], 3
        for v in self.CFG:
            if v == "M":
                layers.append(nn.MaxPool2d(2, 2))
            else:
                layers += [nn.Conv2d(cin, v, 3, padding=1), nn.ReLU(inplace=True)]
                cin = v
        self.features = nn.Sequential(*layers)
        self.classifier = nn.Sequential(
            nn.Linear(512 * 7 * 7, 4096), nn.ReLU(inplace=True), nn.Dropout(),
            nn.Linear(4096, 4096), nn.ReLU(inplace=True), nn.Dropout(),
            nn.Linear(4096, num_classes))

    def forward(self, x):
        x = self.features(x)
        x = F.adaptive_avg_pool2d(x, 7)
        return self.classifier(torch.flatten(x, 1))


# ----------------------------------------------------------------------------- DeepLab-V3+


def _cbr(cin, cout, k=3, stride=1, groups=1, dilation=1, act=True):
    pad = dilation * (k - 1) // 2
    mods = [nn.Conv2d(cin, cout, k, stride, pad, dilation=dilation, groups=groups, bias=False), nn.BatchNorm2d(cout)]
    if act:
        mods.append(nn.ReLU6(inplace=True))
    return nn.Sequential(*mods)


class InvertedResidual(nn.Module):
    def __init__(self, cin, cout, stride, expand, dilation=1):
        super().__init__()
        hidden = cin * expand
        self.use_res = stride == 1 and cin == cout
        mods = []
        if expand != 1:
            mods.append(_cbr(cin, hidden, 1))
        mods += [_cbr(hidden, hidden, 3, stride, groups=hidden, dilation=dilation), _cbr(hidden, cout, 1, act=False)]
        self.conv = nn.Sequential(*mods)

    def forward(self, x):
        y = self.conv(x)
        return x + y if self.use_res else y


class MobileNetV2Backbone(nn.Module):
    """MobileNet-V2 with output stride 16 (last stage dilated), low-level features at /4."""

    # expand, channels, repeats, stride
    CFG = [(1, 16, 1, 1), (6, 24, 2, 2), (6, 32, 3, 2), (6, 64, 4, 2), (6, 96, 3, 1), (6, 160, 3, 1), (6, 320, 1, 1)]

    def __init__(self):
        super().__init__()
        self.stem = _cbr(3, 32, 3, 2)
        layers, cin, stride_total, dilation = [], 32, 2, 1
        self.low_level_idx = None
        for t, c, n, s in self.CFG:
            if stride_total == 16 and s == 2:
                dilation, s = dilation * 2, 1
            for i in range(n):
                layers.append(InvertedResidual(cin, c, s if i == 0 else 1, t, dilation))
                cin = c
            stride_total *= s
            if c == 24:
                self.low_level_idx = len(layers)
        self.layers = nn.ModuleList(layers)
        self.out_channels = cin

    def forward(self, x):
        x = self.stem(x)
        low = None
        for i, m in enumerate(self.layers):
            x = m(x)
            if i + 1 == self.low_level_idx:
                low = x
        return low, x


class ASPP(nn.Module):
    def __init__(self, cin, cout=256, rates=(6, 12, 18)):
        super().__init__()
        self.branches = nn.ModuleList([_conv_bn_relu(cin, cout, 1)] +
                                      [_conv_bn_relu(cin, cout, 3, dilation=r) for r in rates])
        # Image-pooling branch without BN: it sees one value per channel per sample and the
        # training case runs batch 1 (BN would be undefined there).
        self.pool = nn.Sequential(nn.Conv2d(cin, cout, 1), nn.ReLU(inplace=True))
        self.project = _conv_bn_relu(cout * (len(rates) + 2), cout, 1)

    def forward(self, x):
        outs = [b(x) for b in self.branches]
        p = self.pool(F.adaptive_avg_pool2d(x, 1))
        outs.append(F.interpolate(p, size=x.shape[-2:], mode="bilinear", align_corners=False))
        return self.project(torch.cat(outs, 1))


def _conv_bn_relu(cin, cout, k, dilation=1):
    pad = dilation * (k - 1) // 2
    return nn.Sequential(nn.Conv2d(cin, cout, k, padding=pad, dilation=dilation, bias=False), nn.BatchNorm2d(cout),
                         nn.ReLU(inplace=True))


class DeepLabV3Plus(nn.Module):
    def __init__(self, num_classes=21):
        super().__init__()
        self.backbone = MobileNetV2Backbone()
        self.aspp = ASPP(self.backbone.out_channels)
        self.low_proj = _conv_bn_relu(24, 48, 1)
        self.decoder = nn.Sequential(_conv_bn_relu(256 + 48, 256, 3), _conv_bn_relu(256, 256, 3))
        self.cls = nn.Conv2d(256, num_classes, 1)

    def forward(self, x):
        size = x.shape[-2:]
        low, high = self.backbone(x)
        y = self.aspp(high)
        y = F.interpolate(y, size=low.shape[-2:], mode="bilinear", align_corners=False)
        y = self.decoder(torch.cat([y, self.low_proj(low)], 1))
        return F.interpolate(self.cls(y), size=size, mode="bilinear", align_corners=False)


# ----------------------------------------------------------------------------- LSTM


class LSTMSentiment(nn.Module):
    def __init__(self, features=300, hidden=128, num_classes=2):
        super().__init__()
        self.lstm = nn.LSTM(features, hidden, batch_first=True)
        self.fc = nn.Linear(hidden, num_classes)

    def forward(self, x):
        out, _ = self.lstm(x)
        return self.fc(out[:, -1])


# ----------------------------------------------------------------------------- cases


@dataclass
class Case:
    name: str          # e.g. "resnet50-inf"
    test_id: str       # ai-benchmark test number (README.md:57-68)
    model: str
    train: bool
    batch: int
    input_shape: tuple  # per-sample shape
    baseline_native: float   # V100 images/s
    baseline_vgpu: float
    unit: str = "images/s"
    num_classes: int = 1000
    kind: str = "image"      # image | segment | sequence
    factory: object = field(default=None, repr=False)


CASES = [
    Case("resnet50-inf", "1.1", "ResNet-V2-50", False, 50, (3, 346, 346), 135.86, 141.2, factory=resnet_v2_50),
    Case("resnet50-train", "1.2", "ResNet-V2-50", True, 20, (3, 346, 346), 45.24, 43.68, factory=resnet_v2_50),
    Case("resnet152-inf", "2.1", "ResNet-V2-152", False, 10, (3, 256, 256), 110.0, 102.0, factory=resnet_v2_152),
    Case("resnet152-train", "2.2", "ResNet-V2-152", True, 10, (3, 256, 256), 32.67, 30.2, factory=resnet_v2_152),
    Case("vgg16-inf", "3.1", "VGG-16", False, 20, (3, 224, 224), 137.9, 134.2, factory=VGG16),
    Case("vgg16-train", "3.2", "VGG-16", True, 2, (3, 224, 224), 8.62, 8.62, factory=VGG16),
    Case("deeplab-inf", "4.1", "DeepLab", False, 2, (3, 512, 512), 8.97, 8.92, num_classes=21, kind="segment",
         factory=DeepLabV3Plus),
    Case("deeplab-train", "4.2", "DeepLab", True, 1, (3, 384, 384), 4.15, 4.09, num_classes=21, kind="segment",
         factory=DeepLabV3Plus),
    Case("lstm-inf", "5.1", "LSTM", False, 100, (1024, 300), 22.78, 22.32, unit="sequences/s", num_classes=2,
         kind="sequence", factory=LSTMSentiment),
    Case("lstm-train", "5.2", "LSTM", True, 10, (1024, 300), 4.66, 3.96, unit="sequences/s", num_classes=2,
         kind="sequence", factory=LSTMSentiment),
]


def get_case(name):
    for c in CASES:
        if c.name == name:
            return c
    raise KeyError(f"unknown case {name!r}; known: {[c.name for c in CASES]}")


class Runner:
    """One benchmark case bound to a device: ``step()`` runs one full batch.

    Inference: forward only under ``torch.inference_mode``. Training: forward, loss,
    backward and optimizer step. Synthetic inputs/labels are generated once on the
    device (the reference's ai-benchmark also feeds a fixed random batch).

    Defaults are the product's tenant: stock PyTorch at fp32 (the reference's TF
    precision). The tenant is always stock PyTorch-ROCm (MIOpen / hipBLASLt kernels), as
    the reference's benchmark pods run stock TensorFlow.
    """

    def __init__(self, case, device, dtype=torch.float32, batch=None, channels_last=True, seed=0):
        self.case, self.device, self.dtype = case, torch.device(device), dtype
        self.batch = batch or case.batch
        g = torch.Generator(device="cpu").manual_seed(seed)
        torch.manual_seed(seed)
        model = case.factory(num_classes=case.num_classes) if case.kind != "sequence" else case.factory()
        self.image = case.kind in ("image", "segment")
        self.mf = torch.channels_last if (channels_last and self.image) else torch.contiguous_format
        model = model.to(self.device, memory_format=self.mf)
        x = torch.randn((self.batch, *case.input_shape), generator=g)
        if case.kind == "segment":
            y = torch.randint(0, case.num_classes, (self.batch, *case.input_shape[1:]), generator=g)
        else:
            y = torch.randint(0, case.num_classes, (self.batch,), generator=g)
        self.x = x.to(self.device).contiguous(memory_format=self.mf)
        self.y = y.to(self.device)
        if case.train:
            model.train()
            self.opt = torch.optim.SGD(model.parameters(), lr=1e-3, momentum=0.9)
        else:
            model.eval()
            model = model.to(dtype)
            self.x = self.x.to(dtype)
            self.opt = None
        self.model = model

    def capture(self, warmup=3):
        """Capture one step into a HIP graph (torch.cuda.CUDAGraph); later steps replay it
        with a single launch. Inference captures the forward; training captures forward,
        loss, backward and the optimizer step (the "whole network" pattern: gradients are
        None at capture so every replay writes them afresh, autocast runs without its
        weight cache). Warm-up runs on a side stream first so lazy initialisation, MIOpen
        autotuning and optimizer-state creation happen outside the capture."""
        if self.device.type != "cuda":
            raise ValueError("graph capture needs a GPU")
        if self.case.train and self.case.kind == "sequence":
            # Measured on MI355X (ROCm 7.2, PyTorch 2.10): capturing the MIOpen RNN
            # backward kills the process, so recurrent training always runs eagerly.
            raise NotImplementedError("MIOpen RNN training is not HIP-graph capturable")
        cur = torch.cuda.current_stream(self.device)
        s = torch.cuda.Stream(self.device)
        s.wait_stream(cur)
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._eager_step(cache=False)
        cur.wait_stream(s)
        self.graph = torch.cuda.CUDAGraph()
        if self.case.train:
            self.opt.zero_grad(set_to_none=True)
            with torch.cuda.graph(self.graph):
                self.graph_out = self._eager_step(cache=False, zero_grad=False)
        else:
            with torch.inference_mode(), torch.cuda.graph(self.graph):
                self.graph_out = self.model(self.x)
        return self

    def _eager_step(self, cache=True, zero_grad=True):
        if not self.case.train:
            with torch.inference_mode():
                return self.model(self.x)
        with torch.autocast(self.device.type, dtype=self.dtype, enabled=self.dtype != torch.float32,
                            cache_enabled=cache):
            out = self.model(self.x)
            loss = F.cross_entropy(out.float(), self.y)
        if zero_grad:
            self.opt.zero_grad(set_to_none=True)
        loss.backward()
        self.opt.step()
        return loss

    def step(self):
        if getattr(self, "graph", None) is not None:
            self.graph.replay()
            return self.graph_out
        return self._eager_step()

    @property
    def items_per_step(self):
        return self.batch


def build_case(name, device="cuda", **kw):
    return Runner(get_case(name), device, **kw)
