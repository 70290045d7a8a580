#!/usr/bin/env python3
"""MFMA conv with fused epilogue (native/src/kernels/conv_nhwc_mfma.hip) vs the path it
replaces: library convolution (MIOpen/CK, find-mode tuned) followed by the fused
BN+ReLU(+residual) pass. Shapes are every distinct convolution of ResNet-V2-50 inference
at the ai-benchmark 1.1 configuration (batch 50, 346x346) except the 3-channel stem,
with the epilogue it carries.

    python benchmarks/conv_bench.py [--iters 50] [--md-out F] [--json-out F]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

# (label, batch, H, W, Cin, Cout, kernel, stride, pad, epilogue)
SHAPES = [
    ("s1 conv1 (first)", 50, 87, 87, 64, 64, 1, 1, 0, "bn_act"),
    ("s1 conv1", 50, 87, 87, 256, 64, 1, 1, 0, "bn_act"),
    ("s1 conv2 3x3", 50, 87, 87, 64, 64, 3, 1, 1, "bn_act"),
    ("s1 conv3", 50, 87, 87, 64, 256, 1, 1, 0, "residual_sum"),
    ("s1 shortcut", 50, 87, 87, 64, 256, 1, 1, 0, "plain"),
    ("s2 conv1 (first)", 50, 87, 87, 256, 128, 1, 1, 0, "bn_act"),
    ("s2 conv2 3x3/2 (first)", 50, 87, 87, 128, 128, 3, 2, 1, "bn_act"),
    ("s2 conv1", 50, 44, 44, 512, 128, 1, 1, 0, "bn_act"),
    ("s2 conv2 3x3", 50, 44, 44, 128, 128, 3, 1, 1, "bn_act"),
    ("s2 conv3", 50, 44, 44, 128, 512, 1, 1, 0, "residual_sum"),
    ("s2 shortcut 1x1/2", 50, 87, 87, 256, 512, 1, 2, 0, "plain"),
    ("s3 conv1 (first)", 50, 44, 44, 512, 256, 1, 1, 0, "bn_act"),
    ("s3 conv2 3x3/2 (first)", 50, 44, 44, 256, 256, 3, 2, 1, "bn_act"),
    ("s3 conv1", 50, 22, 22, 1024, 256, 1, 1, 0, "bn_act"),
    ("s3 conv2 3x3", 50, 22, 22, 256, 256, 3, 1, 1, "bn_act"),
    ("s3 conv3", 50, 22, 22, 256, 1024, 1, 1, 0, "residual_sum"),
    ("s3 shortcut 1x1/2", 50, 44, 44, 512, 1024, 1, 2, 0, "plain"),
    ("s4 conv1 (first)", 50, 22, 22, 1024, 512, 1, 1, 0, "bn_act"),
    ("s4 conv2 3x3/2 (first)", 50, 22, 22, 512, 512, 3, 2, 1, "bn_act"),
    ("s4 conv1", 50, 11, 11, 2048, 512, 1, 1, 0, "bn_act"),
    ("s4 conv2 3x3", 50, 11, 11, 512, 512, 3, 1, 1, "bn_act"),
    ("s4 conv3", 50, 11, 11, 512, 2048, 1, 1, 0, "residual_sum"),
    ("s4 shortcut 1x1/2", 50, 22, 22, 1024, 2048, 1, 2, 0, "plain"),
]


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
    import torch.nn.functional as F
    from amdvgpu.ops.fused import bn_act, conv_nhwc, conv_weight_2d
    torch.backends.cudnn.benchmark = True
    rows = []
    for label, n, h, w, cin, cout, k, st, pad, epi in SHAPES:
        x = torch.randn(n, cin, h, w, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device="cuda") / (cin * k * k) ** 0.5).to(torch.bfloat16)
        wt = wt.contiguous(memory_format=torch.channels_last)
        w2 = conv_weight_2d(wt)
        oh, ow = (h + 2 * pad - k) // st + 1, (w + 2 * pad - k) // st + 1
        r = torch.randn(n, cout, oh, ow, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        sc = torch.rand(cout, device="cuda") + 0.5
        sh = torch.randn(cout, device="cuda")
        res = epi == "residual_sum"
        conv_only = lambda: F.conv2d(x, wt, stride=st, padding=pad)  # noqa: E731
        with torch.inference_mode():
            if res:
                fused = lambda: conv_nhwc(x, wt, st, pad, sc, sh, r, "relu", write_sum=True, w2d=w2)  # noqa: E731
                lib = lambda: bn_act(conv_only(), sc, sh, r, "relu", write_sum=True)  # noqa: E731
            elif epi == "bn_act":
                fused = lambda: conv_nhwc(x, wt, st, pad, sc, sh, act="relu", w2d=w2)  # noqa: E731
                lib = lambda: bn_act(conv_only(), sc, sh, act="relu")  # noqa: E731
            else:
                fused = lambda: conv_nhwc(x, wt, st, pad, w2d=w2)  # noqa: E731
                lib = conv_only
            t_f, t_l, t_c = timeit(fused, a.iters), timeit(lib, a.iters), timeit(conv_only, a.iters)
            y_f = fused()
            y_l = lib()
            y_f, y_l = (y_f[0], y_l[0]) if res else (y_f, y_l)
            err = (y_f.float() - y_l.float()).abs().max().item()
        m = n * oh * ow
        flops = 2.0 * m * cin * k * k * cout
        nbytes = 2 * (n * h * w * cin + cout * cin * k * k + m * cout * (3 if res else 1))  # x, w, y (+ r, sum)
        rows.append({"layer": label, "M": m, "K": cin * k * k, "N": cout, "epilogue": epi, "fused_us": t_f,
                     "library_conv_plus_epilogue_us": t_l, "library_conv_only_us": t_c,
                     "speedup": t_l / t_f, "fused_TBps": nbytes / t_f / 1e6, "fused_TFLOPs": flops / t_f / 1e6,
                     "max_abs_diff_vs_library": err})
        print(json.dumps(rows[-1]), flush=True)
    # The stem: conv7x7/2 (3 -> 64) + maxpool3x3/2 + first BN + ReLU, one fused kernel
    # (stem_mfma.hip) vs library conv + max-pool + the fused BN+ReLU pass.
    from amdvgpu.ops.fused import stem_pool_bn_act, stem_weight
    x = torch.randn(50, 3, 346, 346, device="cuda").to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    wt = (torch.randn(64, 3, 7, 7, device="cuda") / 147 ** 0.5).to(torch.bfloat16).contiguous(
        memory_format=torch.channels_last)
    w192 = stem_weight(wt)
    sc, sh = torch.rand(64, device="cuda") + 0.5, torch.randn(64, device="cuda")
    with torch.inference_mode():
        fused = lambda: stem_pool_bn_act(x, w192, sc, sh)  # noqa: E731
        conv_only = lambda: F.conv2d(x, wt, stride=2, padding=3)  # noqa: E731
        lib = lambda: bn_act(F.max_pool2d(conv_only(), 3, 2, 1), sc, sh, act="relu")  # noqa: E731
        t_f, t_l, t_c = timeit(fused, a.iters), timeit(lib, a.iters), timeit(conv_only, a.iters)
        err = (fused().float() - lib().float()).abs().max().item()
    m = 50 * 173 * 173
    rows.append({"layer": "stem conv7x7/2 + pool + bn", "M": m, "K": 147, "N": 64, "epilogue": "pool_bn_act",
                 "fused_us": t_f, "library_conv_plus_epilogue_us": t_l, "library_conv_only_us": t_c,
                 "speedup": t_l / t_f, "fused_TBps": 2 * (x.numel() + 50 * 64 * 87 * 87) / t_f / 1e6,
                 "fused_TFLOPs": 2.0 * m * 147 * 64 / t_f / 1e6, "max_abs_diff_vs_library": err})
    print(json.dumps(rows[-1]), flush=True)
    # Projection blocks: conv3 + the 1x1 shortcut as one dual-source GEMM (conv_dual) vs
    # the two-kernel form (shortcut conv, then conv3 with the shortcut as its residual).
    from amdvgpu.ops.fused import conv_dual, conv_dual_weight
    dual_rows = []
    for label, n, h2, c1, c2, s2, cout in (("s1 conv3 + shortcut", 50, 87, 64, 64, 1, 256),
                                           ("s2 conv3 + shortcut/2", 50, 87, 128, 256, 2, 512),
                                           ("s3 conv3 + shortcut/2", 50, 44, 256, 512, 2, 1024),
                                           ("s4 conv3 + shortcut/2", 50, 22, 512, 1024, 2, 2048)):
        h = (h2 - 1) // s2 + 1
        cl = torch.channels_last
        y = torch.randn(n, c1, h, h, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        pre = torch.randn(n, c2, h2, h2, device="cuda").to(torch.bfloat16).contiguous(memory_format=cl)
        w3 = (torch.randn(cout, c1, 1, 1, device="cuda") / c1 ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        ws = (torch.randn(cout, c2, 1, 1, device="cuda") / c2 ** 0.5).to(torch.bfloat16).contiguous(memory_format=cl)
        wcat = conv_dual_weight(w3, ws)
        w3d, wsd = conv_weight_2d(w3), conv_weight_2d(ws)
        with torch.inference_mode():
            dual = lambda: conv_dual(y, pre, wcat, s2)  # noqa: E731
            two = lambda: conv_nhwc(y, w3, 1, 0, residual=conv_nhwc(pre, ws, s2, 0, w2d=wsd), w2d=w3d)  # noqa: E731
            t_d, t_2 = timeit(dual, a.iters), timeit(two, a.iters)
            err = (dual().float() - two().float()).abs().max().item()
        m = n * h * h
        nbytes = 2 * (m * c1 + n * h2 * h2 * c2 + cout * (c1 + c2) + m * cout)
        dual_rows.append({"block": label, "M": m, "K": c1 + c2, "N": cout, "dual_us": t_d, "two_kernels_us": t_2,
                          "speedup": t_2 / t_d, "dual_TBps": nbytes / t_d / 1e6,
                          "dual_TFLOPs": 2.0 * m * (c1 + c2) * cout / t_d / 1e6, "max_abs_diff": err})
        print(json.dumps(dual_rows[-1]), flush=True)
    tot_f = sum(r_["fused_us"] for r_ in rows)
    tot_l = sum(r_["library_conv_plus_epilogue_us"] for r_ in rows)
    md = ["| layer | M | K | N | epilogue | fused MFMA us | library conv + epilogue us | conv alone us | speedup "
          "| fused TB/s | fused TFLOP/s | max abs diff |", "|---|---|---|---|---|---|---|---|---|---|---|---|"]
    for r_ in rows:
        md.append(f"| {r_['layer']} | {r_['M']} | {r_['K']} | {r_['N']} | {r_['epilogue']} | {r_['fused_us']:.1f} | "
                  f"{r_['library_conv_plus_epilogue_us']:.1f} | {r_['library_conv_only_us']:.1f} | "
                  f"{r_['speedup']:.2f}x | {r_['fused_TBps']:.2f} | {r_['fused_TFLOPs']:.0f} | "
                  f"{r_['max_abs_diff_vs_library']:.3g} |")
    md.append(f"| **sum (one of each)** | | | | | {tot_f:.1f} | {tot_l:.1f} | | {tot_l / tot_f:.2f}x | | | |")
    md += ["", "Projection blocks: conv3 + shortcut as one dual-source GEMM vs shortcut conv + conv3 with residual "
           "(both MFMA kernels)", "",
           "| block | M | K | N | dual us | two kernels us | speedup | dual TB/s | dual TFLOP/s | max abs diff |",
           "|---|---|---|---|---|---|---|---|---|---|"]
    for r_ in dual_rows:
        md.append(f"| {r_['block']} | {r_['M']} | {r_['K']} | {r_['N']} | {r_['dual_us']:.1f} | "
                  f"{r_['two_kernels_us']:.1f} | {r_['speedup']:.2f}x | {r_['dual_TBps']:.2f} | "
                  f"{r_['dual_TFLOPs']:.0f} | {r_['max_abs_diff']:.3g} |")
    print("\n".join(md))
    if a.json_out:
        json.dump(rows, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
