#!/usr/bin/env python3
"""Per-call cost of the interception shim on the hot paths (no published reference
number exists). Measures, natively and inside a vGPU (quota only, and
quota + temporal limiter with the bucket effectively unlimited):

* launch     back-to-back tiny kernel launches (torch add_ on 1 element), per-launch us
* graph      hipGraphLaunch of a captured 16-kernel graph, per-replay us
* malloc     hipMalloc + hipFree of 2 MiB through ROCr (bypasses torch's cache), per pair us
* memcpy     hipMemcpyAsync D2D of 4 KiB, per call us

    python benchmarks/hook_overhead.py [--iters 20000]
"""
import argparse
import ctypes
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def worker(iters, out):
    import torch
    x = torch.zeros(1, device="cuda")
    for _ in range(1000):
        x.add_(1)
    torch.cuda.synchronize()
    res = {}
    t0 = time.perf_counter()
    for _ in range(iters):
        x.add_(1)
    torch.cuda.synchronize()
    res["launch_us"] = (time.perf_counter() - t0) / iters * 1e6

    g = torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        x.add_(1)
    torch.cuda.synchronize()
    with torch.cuda.graph(g):
        for _ in range(16):
            x.add_(1)
    g.replay()
    torch.cuda.synchronize()
    n = max(1, iters // 16)
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
    torch.cuda.synchronize()
    res["graph_replay_us"] = (time.perf_counter() - t0) / n * 1e6

    hip = None
    for cand in ("libamdhip64.so", "libamdhip64.so.7", "libamdhip64.so.6"):
        try:
            hip = ctypes.CDLL(cand, mode=ctypes.RTLD_GLOBAL)
            break
        except OSError:
            continue
    p = ctypes.c_void_p()
    m = max(1, iters // 20)
    hip.hipMalloc(ctypes.byref(p), 2 << 20)
    hip.hipFree(p)
    t0 = time.perf_counter()
    for _ in range(m):
        hip.hipMalloc(ctypes.byref(p), 2 << 20)
        hip.hipFree(p)
    res["malloc_free_us"] = (time.perf_counter() - t0) / m * 1e6

    a = torch.empty(4096, dtype=torch.uint8, device="cuda")
    b = torch.empty_like(a)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(iters // 4):
        b.copy_(a)
    torch.cuda.synchronize()
    res["memcpy_us"] = (time.perf_counter() - t0) / (iters // 4) * 1e6
    json.dump(res, open(out, "w"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iters", type=int, default=20000)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--modes", default="", help="comma-separated subset of the modes")
    ap.add_argument("--probe", action="store_true", help="the C++ probe (native/tests/hip_launch_probe.hip) "
                    "instead of the PyTorch worker")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.iters, a.out)
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    modes = {"native": None, "vgpu": dict(mem_limit=64 << 30),
             "vgpu-stats": dict(mem_limit=64 << 30, extra={"VGPU_STATS": "1"}),
             "vgpu-temporal": dict(mem_limit=64 << 30, cu_limit=99, cu_mode="temporal"),
             # diagnostics: the gates made pass-throughs (trampolines stay), the dlsym routing off
             "vgpu-nogate": dict(mem_limit=64 << 30, extra={"VGPU_HOOK_LAUNCH": "0"}),
             "vgpu-nodlsym": dict(mem_limit=64 << 30, extra={"VGPU_HOOK_DLSYM": "0"})}
    if a.modes:
        modes = {m: modes[m] for m in a.modes.split(",")}
    best = {}
    for rep in range(a.repeats):
        for mode, kw in modes.items():
            c = vgpu_env(**kw) if kw else {}
            env = apply_contract(c) if c else dict(os.environ)
            fd, out = tempfile.mkstemp(suffix=".json")
            os.close(fd)
            try:
                if a.probe:
                    from amdvgpu.shim.native import lib_path
                    line = subprocess.check_output([lib_path("hip_launch_probe"), str(a.iters * 5), str(a.iters * 50)],
                                                   env=env, text=True)
                    r = json.loads([l for l in line.splitlines() if l.startswith("{")][-1])
                else:
                    subprocess.check_call([sys.executable, os.path.abspath(__file__), "--worker", "--iters",
                                           str(a.iters), "--out", out], env=env)
                    r = json.load(open(out))
            finally:
                os.unlink(out)
                cleanup_region(c)
            for k, v in r.items():
                best.setdefault(mode, {})[k] = min(v, best.get(mode, {}).get(k, float("inf")))
            print(mode, json.dumps(r), flush=True)
    keys = list(best["native"])
    md = ["| metric (us/call, best of %d) | %s |" % (a.repeats, " | ".join(modes)), "|---|" + "---|" * len(modes)]
    for k in keys:
        md.append(f"| {k} | " + " | ".join(f"{best[m][k]:.3f}" for m in modes) + " |")
    print("\n".join(md))
    if a.json_out:
        json.dump(best, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
