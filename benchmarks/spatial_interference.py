#!/usr/bin/env python3
"""Where does concurrent CU-masked tenancy lose throughput? Runs N tenants on disjoint
CU slices (and, for comparison, unmasked) with two synthetic workloads built from the
calibration kernels:

* spin     compute-only: single-wave workgroups that spin a fixed time (no memory traffic);
           every workgroup of a launch fits on the slice at once
* copy     memory-only: 16 B/lane stream copy of a 1 GiB buffer
* spin-lds compute-only like spin, but each workgroup holds 64 KiB of LDS, so a launch is
           dispatched over many rounds (the shape of a GEMM/conv grid)

Reports per-tenant time for a fixed amount of work, solo vs concurrent.

    python benchmarks/spatial_interference.py [--tenants 4]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def worker(kind, iters, out, go):
    import torch
    from amdvgpu.ops import spin, stream_copy
    if kind == "copy":
        a = torch.empty(1 << 30, dtype=torch.uint8, device="cuda")
        b = torch.empty_like(a)
        fn = lambda: stream_copy(b, a)  # noqa: E731
    elif kind == "spin-lds":
        # 2 workgroups per CU at a time (64 KiB LDS each), 4096 per launch: like a GEMM
        # grid, dispatched over many rounds on a CU slice.
        from amdvgpu.ops import spin_lds
        fn = lambda: spin_lds(4096, 20, 64 << 10)  # noqa: E731
    else:
        fn = lambda: spin(256 * 8, 200)  # noqa: E731
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    open(out + ".ready", "w").close()
    while not os.path.exists(go):
        time.sleep(0.002)
    t0 = time.perf_counter()
    for _ in range(iters):
        fn()
    torch.cuda.synchronize()
    json.dump({"t": time.perf_counter() - t0}, open(out, "w"))


def run(kind, n, masked, iters, solo=False):
    from amdvgpu.plugin.vdevice import cu_partition_range
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    tmp = tempfile.mkdtemp()
    go = os.path.join(tmp, "go")
    procs, outs, cs = [], [], []
    for i in range(1 if solo else n):
        kw = dict(mem_limit=16 << 30)
        if masked and n > 1:
            b, e = cu_partition_range(256, 8, n, i)
            kw.update(cu_limit=100 * (e - b) // 256, cu_range=(b, e))
        c = vgpu_env(**kw)
        out = os.path.join(tmp, f"{i}.json")
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--worker", "--kind", kind,
                                       "--iters", str(iters), "--out", out, "--go", go], env=apply_contract(c)))
        outs.append(out)
        cs.append(c)
    try:
        while not all(os.path.exists(o + ".ready") for o in outs):
            if any(p.poll() not in (None, 0) for p in procs):
                raise SystemExit("tenant failed")
            time.sleep(0.02)
        open(go, "w").close()
        for p in procs:
            if p.wait(timeout=600) != 0:
                raise SystemExit("tenant failed")
        return [json.load(open(o))["t"] for o in outs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for c in cs:
            cleanup_region(c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--tenants", type=int, default=4)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--kind", default="spin")
    ap.add_argument("--iters", type=int, default=200)
    ap.add_argument("--out")
    ap.add_argument("--go")
    ap.add_argument("--md-out")
    ap.add_argument("--kinds", default="spin,copy,spin-lds")
    a = ap.parse_args()
    if a.worker:
        return worker(a.kind, a.iters, a.out, a.go)
    n = a.tenants
    rows = []
    kinds = [(k, {"spin": 200, "copy": 50, "spin-lds": 20}[k]) for k in a.kinds.split(",")]
    for kind, iters in kinds:
        for masked in (True, False):
            solo = run(kind, n, masked, iters, solo=True)[0]
            conc = run(kind, n, masked, iters)
            rows.append({"kind": kind, "masked": masked, "solo_s": solo, "concurrent_s": conc,
                         "slowdown": max(conc) / solo})
            print(json.dumps(rows[-1]), flush=True)
    md = [f"| workload | CU slices ({n} tenants) | solo s | concurrent s (max) | slowdown |", "|---|---|---|---|---|"]
    md += [f"| {r['kind']} | {'disjoint masks' if r['masked'] else 'none (shared)'} | {r['solo_s']:.3f} | "
           f"{max(r['concurrent_s']):.3f} | {r['slowdown']:.2f}x |" for r in rows]
    print("\n".join(md))
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
