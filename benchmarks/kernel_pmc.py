#!/usr/bin/env python3
"""Workload for per-kernel hardware-counter passes (rocprofv3 --pmc) over the hand-written
gfx950 kernels at ResNet-V2-50 inference shapes (batch 50, 346x346): the fused stem, a
stage-1 3x3 conv (implicit GEMM, BN+ReLU epilogue), a stage-1 conv3 (1x1, sum-only
epilogue) and a stage-1 conv1 with the BN+ReLU prologue; or (--set conv3x3) the 3x3
convs of all four stages. Each runs --iters times.

    rocprofv3 --pmc <counters> --kernel-trace --output-format csv -d OUT -o p1 -- \\
        python3 benchmarks/kernel_pmc.py
    python tools/pmc_summary.py --all-counters p1=OUT/**/p1_counter_collection.csv
"""
import argparse
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=5)
    ap.add_argument("--set", default="mixed", choices=["mixed", "conv3x3"],
                    help="conv3x3: the four stages' 3x3 convs (BN+ReLU epilogue) instead")
    a = ap.parse_args()
    import torch
    from amdvgpu.ops.fused import conv_nhwc, stem_pool_bn_act, stem_weight
    cl = torch.channels_last
    dev = "cuda"
    x = torch.randn(50, 3, 346, 346, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w7 = (torch.randn(64, 3, 7, 7, device=dev) / 147 ** 0.5).to(torch.bfloat16)
    w192 = stem_weight(w7)
    s64, t64 = torch.rand(64, device=dev) + 0.5, torch.randn(64, device=dev)
    s256, t256 = torch.rand(256, device=dev) + 0.5, torch.randn(256, device=dev)
    y64 = torch.randn(50, 64, 87, 87, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    x256 = torch.randn(50, 256, 87, 87, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
    w33 = (torch.randn(64, 64, 3, 3, device=dev) / 576 ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
    w3 = (torch.randn(256, 64, 1, 1, device=dev) / 8).to(torch.bfloat16).contiguous(memory_format=cl)
    w1 = (torch.randn(64, 256, 1, 1, device=dev) / 16).to(torch.bfloat16).contiguous(memory_format=cl)
    if a.set == "conv3x3":
        layers = []
        for c, hw in ((64, 87), (128, 44), (256, 22), (512, 11)):
            xi = torch.randn(50, c, hw, hw, device=dev).to(torch.bfloat16).contiguous(memory_format=cl)
            wi = (torch.randn(c, c, 3, 3, device=dev) / (9 * c) ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
            layers.append((xi, wi, torch.rand(c, device=dev) + 0.5, torch.randn(c, device=dev)))
        with torch.inference_mode():
            for _ in range(a.iters):
                for xi, wi, si, ti in layers:
                    conv_nhwc(xi, wi, 1, 1, si, ti, act="relu")
            torch.cuda.synchronize()
        print("kernel_pmc done", flush=True)
        return
    with torch.inference_mode():
        for _ in range(a.iters):
            stem_pool_bn_act(x, w192, s64, t64)
            conv_nhwc(y64, w33, 1, 1, s64, t64, act="relu")
            conv_nhwc(y64, w3, residual=x256)
            conv_nhwc(x256, w1, scale=s64, shift=t64, act="relu", prologue=(s256, t256))
        torch.cuda.synchronize()
    print("kernel_pmc done", flush=True)


if __name__ == "__main__":
    main()
