#!/usr/bin/env python3
"""Fused BN+ReLU(+residual) HIP epilogue vs the eager PyTorch sequence it replaces:
achieved HBM bandwidth per shape (bytes = inputs + outputs, counted once).

    python benchmarks/op_bench.py [--iters 50]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# ResNet-V2-50 at 346x346, batch 50: activation shapes at each stage boundary / inside blocks
SHAPES = [(50, 64, 87, 87), (50, 256, 87, 87), (50, 128, 44, 44), (50, 512, 44, 44), (50, 256, 22, 22),
          (50, 1024, 22, 22), (50, 2048, 11, 11)]


def timeit(fn, iters):
    import torch
    for _ in range(3):
        fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(iters):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / iters * 1000.0  # us


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=50)
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    import torch
    import torch.nn as nn
    from amdvgpu.ops.fused import bn_act, bn_scale_shift
    rows = []
    for shape in SHAPES:
        N, C, H, W = shape
        x = torch.randn(shape, device="cuda", dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        r = torch.randn_like(x)
        bn = nn.BatchNorm2d(C).cuda().eval().to(torch.bfloat16)
        sc, sh = bn_scale_shift(bn)
        nbytes = x.numel() * 2
        t_plain = timeit(lambda: bn_act(x, sc, sh), a.iters)
        t_res = timeit(lambda: bn_act(x, sc, sh, r, write_sum=True), a.iters)
        with torch.inference_mode():
            t_eager_plain = timeit(lambda: torch.relu(bn(x)), a.iters)
            t_eager_res = timeit(lambda: torch.relu(bn(x + r)), a.iters)
        rows.append({"shape": shape, "MB": nbytes / 1e6,
                     "fused_us": t_plain, "fused_GBps": 2 * nbytes / t_plain / 1e3,
                     "eager_us": t_eager_plain,
                     "fused_res_us": t_res, "fused_res_GBps": 4 * nbytes / t_res / 1e3,
                     "eager_res_us": t_eager_res})
        print(json.dumps(rows[-1]), flush=True)
    md = ["| shape (NCHW, bf16 NHWC) | MB | fused bn+relu us | GB/s | eager us | fused add+bn+relu (+sum) us | GB/s | eager us |",
          "|---|---|---|---|---|---|---|---|"]
    for r_ in rows:
        md.append(f"| {r_['shape']} | {r_['MB']:.0f} | {r_['fused_us']:.1f} | {r_['fused_GBps']:.0f} | "
                  f"{r_['eager_us']:.1f} | {r_['fused_res_us']:.1f} | {r_['fused_res_GBps']:.0f} | "
                  f"{r_['eager_res_us']:.1f} |")
    print("\n".join(md))
    if a.json_out:
        json.dump(rows, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
