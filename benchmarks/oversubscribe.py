#!/usr/bin/env python3
"""Virtual device memory (BASELINE.json config 4): one vGPU whose quota exceeds the
MI355X's 288 GiB of HBM. The tenant pins a large HBM-resident ballast and then trains the
LSTM (ai-benchmark test 5.2, batch 10, 1024 x 300); allocations past the tenant's HBM
share are served from pinned host memory by the shim (VGPU_DEVICE_HBM_LIMIT +
VGPU_OVERSUBSCRIBE). Reports quota seen by the process, bytes spilled, and training
throughput with / without spill. (The reference switches *all* allocations to CUDA
managed memory instead)

    python benchmarks/oversubscribe.py [--quota-gib 320] [--ballast-gib 270]
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
GiB = 1 << 30


def worker(case, ballast_gib, steps, warmup, out):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = os.environ.get("VGPU_BENCH_TUNE", "1") == "1"  # MIOpen find mode
    from amdvgpu.shim.region import Region
    free, total = torch.cuda.mem_get_info(0)
    ballast = []
    for _ in range(ballast_gib):
        ballast.append(torch.empty(GiB, dtype=torch.uint8, device="cuda"))
    torch.cuda.synchronize()
    r = Runner(get_case(case), "cuda:0")
    for _ in range(warmup):
        r.step()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    ms = (time.perf_counter() - t0) * 1000 / steps
    dev = Region(os.environ["VGPU_SHARED_CACHE"]).device(0) if os.environ.get("VGPU_SHARED_CACHE") else {}
    json.dump({"total": total, "ms_per_batch": ms, "throughput": r.batch * 1000 / ms,
               "spilled": dev.get("spilled", 0), "used": dev.get("used", 0), "ballast_gib": ballast_gib},
              open(out, "w"))


def run(quota_gib, hbm_gib, ballast_gib, case, steps, warmup):
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    c = vgpu_env(mem_limit=quota_gib * GiB, oversubscribe=True,
                 extra={"VGPU_DEVICE_HBM_LIMIT_0": f"{hbm_gib * 1024}m"})
    fd, out = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    try:
        subprocess.check_call([sys.executable, os.path.abspath(__file__), "--worker", "--case", case,
                               "--ballast-gib", str(ballast_gib), "--steps", str(steps), "--warmup", str(warmup),
                               "--out", out], env=apply_contract(c))
        return json.load(open(out))
    finally:
        os.unlink(out)
        cleanup_region(c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--quota-gib", type=int, default=320)
    ap.add_argument("--hbm-gib", type=int, default=272)
    ap.add_argument("--ballast-gib", type=int, default=271)
    ap.add_argument("--case", default="lstm-train")
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--json-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.case, a.ballast_gib, a.steps, a.warmup, a.out)
    res = {"resident": run(a.quota_gib, a.hbm_gib, 0, a.case, a.steps, a.warmup),
           "spilled": run(a.quota_gib, a.hbm_gib, a.ballast_gib, a.case, a.steps, a.warmup)}
    for k, v in res.items():
        print(k, json.dumps(v), flush=True)
    if a.json_out:
        json.dump(res, open(a.json_out, "w"), indent=1)


if __name__ == "__main__":
    main()
