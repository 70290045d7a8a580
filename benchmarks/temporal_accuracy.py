#!/usr/bin/env python3
"""Temporal compute limit: achieved share vs configured limit, on stock workloads.

Each tenant is a separate process (its own vGPU region, as separate containers would
be) running a stock PyTorch-ROCm workload for a fixed wall time; the achieved share is
its throughput divided by the same workload's native (unlimited, alone) throughput.
Measured for one tenant alone and for two identical tenants running concurrently (each
in its own vGPU with the same limit). The reference publishes no accuracy for its
token bucket; round 1 measured 29/44/62 % for 25/50/75 %
(profiles/r1l/temporal.md).

Workloads: ``resnet50`` (ai-benchmark 1.1: ResNet-V2-50 inference, batch 50, 346², fp32,
stock PyTorch/MIOpen), ``spin`` (calibration kernel: 2048 single-wave workgroups of
500 µs — a GPU-bound launch stream with no host gaps).

    python benchmarks/temporal_accuracy.py [--workload resnet50] [--limits 10,25,50,75,90]
                                           [--tenants 1,2] [--seconds 4]
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


def worker(workload, seconds, sync_every, out, go, batch=0):
    import torch
    if workload == "resnet50":
        from amdvgpu.models.aibench import Runner, get_case
        torch.backends.cudnn.benchmark = True
        r = Runner(get_case("resnet50-inf"), "cuda:0", dtype=torch.float32, batch=batch or None)
        step, items = r.step, r.batch
    else:
        from amdvgpu.ops import spin
        step, items = (lambda: spin(2048, 500)), 1
    for _ in range(5):
        step()
    torch.cuda.synchronize()
    open(out + ".ready", "w").close()
    while go and not os.path.exists(go):
        time.sleep(0.002)
    stats0 = _region_stats()
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        step()
        n += 1
        if n % sync_every == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    res = {"steps": n, "seconds": dt, "throughput": n * items / dt}
    stats1 = _region_stats()
    if stats0 and stats1:
        # The container's charged share of the GPU's time over the run, and the time its
        # launches spent blocked at the GPU-time gate (this process's slot).
        res["charged_pct"] = 100.0 * (stats1["charged_ns"] - stats0["charged_ns"]) / max(
            1, stats1["wall_ns"] - stats0["wall_ns"])
        res["throttle_pct"] = 100.0 * (stats1["throttle_ns"] - stats0["throttle_ns"]) / (dt * 1e9)
    json.dump(res, open(out, "w"))


def _region_stats():
    """charged_ns / wall_ns of device 0 and this process's throttle_ns, from the region of
    the container the worker runs in (None outside a vGPU or with a foreign layout)."""
    path = os.environ.get("VGPU_SHARED_CACHE")
    if not path:
        return None
    try:
        from amdvgpu.shim.region import Region
        with Region(path) as r:
            d = r.device(0)
            mine = [p for p in r.procs() if p["pid"] == os.getpid()]
            return {"charged_ns": d["charged_ns"], "wall_ns": d["wall_ns"],
                    "throttle_ns": mine[0]["throttle_ns"] if mine else 0}
    except Exception:
        return None


def run_tenants(workload, contracts, seconds, sync_every, batch=0, shim=None, full=False):
    """Starts len(contracts) tenants (None = native), releases them together, returns
    each one's throughput (with ``full``, each one's result: throughput and, in a vGPU,
    charged_pct / throttle_pct). ``shim`` preloads another build of the shim (A/B runs)."""
    from amdvgpu.shim.launcher import apply_contract, cleanup_region
    tmp = tempfile.mkdtemp(prefix="tacc-")
    go = os.path.join(tmp, "go")
    procs, outs = [], []
    for i, c in enumerate(contracts):
        out = os.path.join(tmp, f"t{i}.json")
        env = apply_contract(c, shim=shim) if c else dict(os.environ)
        cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--workload", workload, "--seconds",
               str(seconds), "--sync-every", str(sync_every), "--out", out, "--go", go, "--batch", str(batch)]
        procs.append(subprocess.Popen(cmd, env=env))
        outs.append(out)
    try:
        deadline = time.time() + 600
        while not all(os.path.exists(o + ".ready") for o in outs):
            if any(p.poll() not in (None, 0) for p in procs) or time.time() > deadline:
                raise SystemExit("a tenant failed before the start barrier")
            time.sleep(0.02)
        open(go, "w").close()
        for p in procs:
            if p.wait(timeout=600) != 0:
                raise SystemExit("a tenant failed")
        res = [json.load(open(o)) for o in outs]
        return res if full else [r["throughput"] for r in res]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
        for c in contracts:
            if c:
                cleanup_region(c)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="resnet50", choices=["resnet50", "spin"])
    ap.add_argument("--limits", default="10,25,50,75,90")
    ap.add_argument("--tenants", default="1,2")
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--sync-every", type=int, default=8)
    ap.add_argument("--batch", type=int, default=0, help="resnet50 batch (default: the case's 50; small = light tenant)")
    ap.add_argument("--extra", default="", help="extra contract env, K=V[,K=V] (e.g. VGPU_LIMITER_WINDOW_MS=120)")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--go")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.workload, a.seconds, a.sync_every, a.out, a.go, a.batch)
    from amdvgpu.shim.launcher import vgpu_env
    native = run_tenants(a.workload, [None], a.seconds, a.sync_every, a.batch)[0]
    print(json.dumps({"native": native}), flush=True)
    rows = []
    for n in [int(x) for x in a.tenants.split(",")]:
        for lim in [int(x) for x in a.limits.split(",")]:
            extra = dict(kv.split("=", 1) for kv in a.extra.split(",") if kv)
            cs = [vgpu_env(cu_limit=lim, cu_mode="temporal", mem_limit=64 << 30, extra=extra) for _ in range(n)]
            full = run_tenants(a.workload, cs, a.seconds, a.sync_every, a.batch, full=True)
            got = [r["throughput"] for r in full]
            ach = [100.0 * g / native for g in got]
            rows.append({"tenants": n, "limit_pct": lim, "throughput": got, "achieved_pct": ach,
                         "charged_pct": [r.get("charged_pct") for r in full],
                         "throttle_pct": [r.get("throttle_pct") for r in full],
                         "max_error_pts": max(abs(x - lim) for x in ach)})
            print(json.dumps(rows[-1]), flush=True)
    label = a.workload + (f" b={a.batch}" if a.batch else "") + (f" [{a.extra}]" if a.extra else "")
    md = [f"# temporal limit accuracy — {label} (native {native:.1f}/s, {a.seconds:.0f} s per point)", "",
          "| tenants | limit % | achieved % (per tenant) | max error (pts) | charged % of GPU time |",
          "|---|---|---|---|---|"]
    for r in rows:
        ch = " / ".join("-" if x is None else f"{x:.1f}" for x in r["charged_pct"])
        md.append(f"| {r['tenants']} | {r['limit_pct']} | {' / '.join(f'{x:.1f}' for x in r['achieved_pct'])} | "
                  f"{r['max_error_pts']:.1f} | {ch} |")
    print("\n".join(md))
    if a.json_out:
        json.dump({"workload": a.workload, "native": native, "rows": rows}, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
