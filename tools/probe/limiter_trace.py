#!/usr/bin/env python3
"""Where does a temporally limited tenant lose throughput? Runs the bench's tenant
(ResNet-V2-50 inference, b=50, fp32, stock PyTorch; the timed loop launches without
per-step syncs, like bench.py) inside a temporal vGPU at several limits while the parent
samples the limiter's state in the shared region every millisecond.

Per limit it reports: ms/step; the GPU time the limiter charged per step (KFD-occupancy
based); charged / wall over the timed window (what the limiter granted); and the credit
trace (JSON) for plotting. If charged-per-step stays at the unlimited value while ms/step
exceeds (native ms/step / limit), the loss is in the grant (gate dynamics); if
charged-per-step grows, the GPU does the same work less efficiently when duty-cycled.

    python tools/probe/limiter_trace.py [--limits 99,50,25,10] [--steps 60] [--out F]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def tenant(steps, warmup, sync_every, marks):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = True
    r = Runner(get_case("resnet50-inf"), "cuda:0", dtype=torch.float32)
    for _ in range(warmup):
        r.step()
    torch.cuda.synchronize()
    t0 = time.time()
    open(marks + ".t0", "w").write(repr(t0))
    for i in range(steps):
        r.step()
        if sync_every and (i + 1) % sync_every == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    t1 = time.time()
    open(marks, "w").write(json.dumps({"t0": t0, "t1": t1, "ms_per_step": (t1 - t0) * 1000 / steps}))


def run_limit(limit, steps, warmup, sync_every, window_ms=0):
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    from amdvgpu.shim.region import Region
    tmp = tempfile.mkdtemp(prefix="ltrace-")
    marks = os.path.join(tmp, "marks.json")
    region = os.path.join(tmp, "region.cache")
    extra = {"VGPU_LIMITER_WINDOW_MS": str(window_ms)} if window_ms else None
    c = vgpu_env(mem_limit=72 << 30, cu_limit=limit, cu_mode="temporal", shared_cache=region, extra=extra)
    cmd = [sys.executable, os.path.abspath(__file__), "--tenant", "--steps", str(steps), "--warmup", str(warmup),
           "--sync-every", str(sync_every), "--marks", marks]
    p = subprocess.Popen(cmd, env=apply_contract(c))
    trace, stop = [], threading.Event()

    def sample():
        while not os.path.exists(region) and not stop.is_set():
            time.sleep(0.01)
        time.sleep(0.5)
        with Region(region) as r:
            while not stop.is_set():
                d = r.device(0)
                trace.append((time.time(), d["credit_ns"], d["charged_ns"], d["wall_ns"]))
                time.sleep(0.001)

    th = threading.Thread(target=sample, daemon=True)
    th.start()
    rc = p.wait(timeout=900)
    stop.set()
    th.join()
    cleanup_region(c)
    if rc:
        raise SystemExit(f"tenant failed at limit {limit}")
    m = json.load(open(marks))
    win = [s for s in trace if m["t0"] <= s[0] <= m["t1"]]
    charged = (win[-1][2] - win[0][2]) / 1e6 if len(win) > 1 else 0.0
    wall = (win[-1][0] - win[0][0]) * 1000 if len(win) > 1 else 0.0
    credits = [s[1] / 1e6 for s in win]
    return {"limit": limit, "window_ms": window_ms, "ms_per_step": m["ms_per_step"], "charged_ms_per_step": charged / steps,
            "granted_frac": charged / wall if wall else None, "credit_min_ms": min(credits) if credits else None,
            "credit_max_ms": max(credits) if credits else None, "samples": len(win),
            "trace": [(round(s[0] - m["t0"], 4), round(s[1] / 1e6, 3), round((s[2] - win[0][2]) / 1e6, 3))
                      for s in win[::4]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--limits", default="99,50,25,10")
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--sync-every", type=int, default=0)
    ap.add_argument("--windows", default="0", help="VGPU_LIMITER_WINDOW_MS values (0 = the shim's default)")
    ap.add_argument("--tenant", action="store_true")
    ap.add_argument("--marks")
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    if a.tenant:
        return tenant(a.steps, a.warmup, a.sync_every, a.marks)
    rows = []
    windows = [int(x) for x in a.windows.split(",")]
    for w in windows:
        for lim in [int(x) for x in a.limits.split(",")]:
            if lim >= 99 and w != windows[0]:
                continue  # the unlimited reference row once
            r = run_limit(lim, a.steps, a.warmup, a.sync_every, w)
            rows.append(r)
            print(json.dumps({k: v for k, v in r.items() if k != "trace"}), flush=True)
    base = rows[0]
    print(f"| window ms | limit % | ms/step | expected ms/step ({base['limit']} % row / limit) | charged ms/step | "
          "granted | throughput vs expected |")
    print("|---|---|---|---|---|---|---|")
    for r in rows:
        exp = base["ms_per_step"] * base["limit"] / r["limit"]
        print(f"| {r['window_ms'] or 'default'} | {r['limit']} | {r['ms_per_step']:.2f} | {exp:.2f} | "
              f"{r['charged_ms_per_step']:.2f} | {(r['granted_frac'] or 0) * 100:.1f} % | "
              f"{exp / r['ms_per_step']:.3f} |")
    if a.out:
        json.dump(rows, open(a.out, "w"))


if __name__ == "__main__":
    main()
