#!/usr/bin/env python3
"""Concurrent-vGPU scaling curve on one MI355X: N tenants (N = 1, 2, 4, 8) each running
the same workload in its own vGPU, started together; reports per-tenant and aggregate
throughput. This is the reference's "vGPU+VDM high load" column (4 containers on 2 GPUs,
BASELINE.md) generalised to the MI355X's tenant counts.

Policies:
* spatial   tenant i of N gets quota HBM/N and the i-th disjoint XCD-balanced CU slice
            (what the plugin hands out with --device-split-count=N)
* shared    quota HBM/N, no CU limit: tenants time-share all 256 CUs (hardware
            scheduling between queues)
* spatial-interleave  same slices in the plain interleaved mask layout (every tenant
            on every SE) instead of the default SE-major layout
* vdm       the reference's "virtual device memory" setting: quota 1.8 x HBM/N with
            oversubscription (HBM share HBM/N, rest spills), CU limit 100*1/N spatial

    python benchmarks/vgpu_scaling.py [--case resnet50-inf] [--tenants 1,2,4,8] [--policy spatial,shared]
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
HBM = 309220868096


def worker(case_name, steps, warmup, out, go_file):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = os.environ.get("VGPU_BENCH_TUNE", "1") == "1"  # MIOpen find mode
    case = get_case(case_name)
    r = Runner(case, "cuda:0")
    for _ in range(warmup):
        r.step()
    torch.cuda.synchronize()
    open(out + ".ready", "w").close()
    while not os.path.exists(go_file):
        time.sleep(0.005)
    t0 = time.perf_counter()
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    json.dump({"ms_per_batch": (t1 - t0) * 1000 / steps, "t0": t0, "t1": t1, "batch": case.batch,
               "throughput": case.batch * steps / (t1 - t0)}, open(out, "w"))


def run_point(case, n, policy, steps, warmup, solo=False):
    from amdvgpu.plugin.vdevice import cu_partition_range
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    tmp = tempfile.mkdtemp(prefix="scal-")
    go = os.path.join(tmp, "go")
    procs, contracts, outs = [], [], []
    for i in range(1 if solo else n):
        kw = dict(mem_limit=HBM // n)
        if policy == "vdm":
            kw = dict(mem_limit=int(HBM * 1.8 / n), oversubscribe=True,
                      extra={"VGPU_DEVICE_HBM_LIMIT_0": f"{HBM // n >> 20}m"})
        if policy in ("spatial", "spatial-interleave", "spatial-q1", "vdm") and n > 1:
            b, e = cu_partition_range(256, 8, n, i)
            kw.update(cu_limit=100 * (e - b) // 256, cu_range=(b, e))
        if policy == "spatial-q1":
            kw["extra"] = dict(kw.get("extra") or {}, GPU_MAX_HW_QUEUES="1")
        if policy == "spatial-interleave":
            kw["extra"] = dict(kw.get("extra") or {}, VGPU_CU_LAYOUT="interleave")
        c = vgpu_env(**kw)
        out = os.path.join(tmp, f"t{i}.json")
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--case", case, "--steps", str(steps),
               "--warmup", str(warmup), "--out", out, "--go", go]
        procs.append(subprocess.Popen(cmd, env=apply_contract(c)))
        contracts.append(c)
        outs.append(out)
    try:
        deadline = time.time() + 600
        while not all(os.path.exists(o + ".ready") for o in outs):
            if any(p.poll() not in (None, 0) for p in procs) or time.time() > deadline:
                raise SystemExit("a tenant failed before the start barrier")
            time.sleep(0.05)
        open(go, "w").close()
        for p in procs:
            if p.wait(timeout=900) != 0:
                raise SystemExit("a tenant failed")
        res = [json.load(open(o)) for o in outs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for c in contracts:
            cleanup_region(c)
    span = max(r["t1"] for r in res) - min(r["t0"] for r in res)
    agg = sum(r["batch"] * steps for r in res) / span
    return {"tenants": n, "policy": policy + ("-solo" if solo else ""), "aggregate_throughput": agg,
            "per_tenant": [r["throughput"] for r in res], "per_tenant_ms": [r["ms_per_batch"] for r in res]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="resnet50-inf")
    ap.add_argument("--tenants", default="1,2,4,8")
    ap.add_argument("--policy", default="spatial,shared")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--solo", action="store_true", help="run only tenant 0 of each N (its slice alone)")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--go")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.case, a.steps, a.warmup, a.out, a.go)
    rows = []
    for pol in a.policy.split(","):
        for n in [int(x) for x in a.tenants.split(",")]:
            r = run_point(a.case, n, pol, a.steps, a.warmup, solo=a.solo)
            rows.append(r)
            print(json.dumps(r), flush=True)
    base = {r["policy"]: r["aggregate_throughput"] for r in rows if r["tenants"] == 1}
    for r in rows:
        base.setdefault(r["policy"], rows[0]["aggregate_throughput"])
    md = [f"# concurrent vGPUs on one MI355X — {a.case}", "",
          "| policy | tenants | aggregate | vs 1 tenant | per-tenant (min..max) |", "|---|---|---|---|---|"]
    for r in rows:
        pt = r["per_tenant"]
        md.append(f"| {r['policy']} | {r['tenants']} | {r['aggregate_throughput']:.1f} | "
                  f"{r['aggregate_throughput'] / base[r['policy']]:.2f}x | {min(pt):.1f} .. {max(pt):.1f} |")
    print("\n".join(md))
    if a.json_out:
        json.dump(rows, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
