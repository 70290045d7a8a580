#!/usr/bin/env python3
"""Temporal (reference-parity) compute limit: achieved share vs configured limit.

A saturating workload (single-wave workgroups spinning a fixed time, a full chip wave
per launch) runs natively and inside a vGPU with VGPU_CU_MODE=temporal at several
limits; the achieved share is native_time / limited_time over a fixed amount of work.
The reference's token bucket has no published accuracy; its grid-block tokens refill
every 120 ms from NVML utilisation.

    python benchmarks/temporal_accuracy.py [--limits 25,50,75] [--seconds 3]
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


def worker(launches, spin_us, out):
    import torch
    from amdvgpu.ops import spin
    spin(256 * 32, 100)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(launches):
        spin(256 * 32, spin_us)
        if i % 64 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    json.dump({"t": time.perf_counter() - t0}, open(out, "w"))


def run(launches, spin_us, contract):
    from amdvgpu.shim.launcher import apply_contract, cleanup_region
    fd, out = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    env = apply_contract(contract) if contract else dict(os.environ)
    try:
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--worker", "--launches", str(launches),
                               "--spin-us", str(spin_us), "--out", out], env=env)
        return json.load(open(out))["t"]
    finally:
        os.unlink(out)
        if contract:
            cleanup_region(contract)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--limits", default="25,50,75")
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--spin-us", type=int, default=500)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--launches", type=int, default=0)
    ap.add_argument("--out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.launches, a.spin_us, a.out)
    from amdvgpu.shim.launcher import vgpu_env
    probe = run(200, a.spin_us, None)
    launches = max(200, int(200 * a.seconds / probe))
    base = run(launches, a.spin_us, None)
    rows = []
    for lim in [int(x) for x in a.limits.split(",")]:
        t = run(launches, a.spin_us, vgpu_env(cu_limit=lim, cu_mode="temporal"))
        rows.append({"limit_pct": lim, "native_s": base, "limited_s": t, "achieved_pct": 100.0 * base / t})
        print(json.dumps(rows[-1]), flush=True)
    md = ["| limit % | native s | limited s | achieved % |", "|---|---|---|---|"]
    md += [f"| {r['limit_pct']} | {r['native_s']:.2f} | {r['limited_s']:.2f} | {r['achieved_pct']:.1f} |"
           for r in rows]
    print("\n".join(md))
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
