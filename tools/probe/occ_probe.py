#!/usr/bin/env python3
"""Probe of KFD's per-process cu_occupancy as a utilisation signal for the temporal limiter.

Measures, on one MI355X: the cost of one sysfs read, and the fraction of samples with
resident waves (busy) for (a) an idle process, (b) a saturating spin workload, (c) a 50 %
duty-cycled spin workload, (d) stock fp32 ResNet-50 inference, (e) two concurrent spinners.

    python tools/probe/occ_probe.py --out gpurun_out/occ_probe.json
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)

CHILD = r"""
import os, sys, time
sys.path.insert(0, %r)
import torch
from amdvgpu.ops import spin
kind = sys.argv[1]
secs = float(sys.argv[2])
x = torch.zeros(1, device="cuda"); torch.cuda.synchronize()
if kind == "resnet":
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = True
    r = Runner(get_case("resnet50-inf"), "cuda:0", dtype=torch.float32)
    for _ in range(5): r.step()
    torch.cuda.synchronize()
print("READY", flush=True)
t0 = time.time()
n = 0
while time.time() - t0 < secs:
    if kind == "idle":
        time.sleep(0.01)
    elif kind == "spin":
        spin(2048, 500); n += 1
        if n %% 16 == 0: torch.cuda.synchronize()
    elif kind == "duty":
        t = time.time()
        for _ in range(10): spin(2048, 500)
        torch.cuda.synchronize()
        busy = time.time() - t
        time.sleep(busy)
    elif kind == "resnet":
        r.step(); n += 1
        if n %% 4 == 0: torch.cuda.synchronize()
torch.cuda.synchronize()
print("DONE", n, flush=True)
""" % REPO


def gpu_id():
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")):
        try:
            v = int(open(p).read().strip() or 0)
        except OSError:
            continue
        if v:
            return v
    raise SystemExit("no GPU node in KFD topology")


def kfd_pids():
    return {int(d) for d in os.listdir("/sys/class/kfd/kfd/proc") if d.isdigit()}


def start(kind, secs):
    """Starts a workload child; returns (Popen, host pid) — sysfs shows host-namespace PIDs,
    so the child's KFD entry is found by diffing the KFD process list around its start."""
    before = kfd_pids()
    p = subprocess.Popen([sys.executable, "-c", CHILD, kind, str(secs)], stdout=subprocess.PIPE, text=True)
    line = p.stdout.readline()
    assert line.startswith("READY"), line
    new = sorted(kfd_pids() - before)
    print(f"{kind}: pid {p.pid} new KFD pids {new}", flush=True)
    p.hostpid = new[0] if len(new) == 1 else (p.pid if p.pid in kfd_pids() else -1)
    return p


def sample(pids, gid, secs):
    paths = [f"/sys/class/kfd/kfd/proc/{p}/stats_{gid}/cu_occupancy" for p in pids]
    vals = [[] for _ in pids]
    lat = []
    t_end = time.perf_counter() + secs
    while time.perf_counter() < t_end:
        for i, path in enumerate(paths):
            t = time.perf_counter()
            try:
                with open(path) as f:
                    v = int(f.read().strip() or -1)
            except OSError:
                v = -1
            lat.append(time.perf_counter() - t)
            vals[i].append(v)
    lat.sort()
    out = {"reads": len(lat), "lat_us_p50": lat[len(lat) // 2] * 1e6, "lat_us_p99": lat[int(len(lat) * .99)] * 1e6}
    for i, v in enumerate(vals):
        ok = [x for x in v if x >= 0]
        out[f"p{i}_busy_frac"] = sum(1 for x in ok if x > 0) / max(1, len(ok))
        out[f"p{i}_mean_occ"] = sum(ok) / max(1, len(ok))
        out[f"p{i}_max_occ"] = max(ok) if ok else -1
        out[f"p{i}_errors"] = len(v) - len(ok)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/occ_probe.json")
    ap.add_argument("--secs", type=float, default=2.0)
    a = ap.parse_args()
    gid = gpu_id()
    res = {"gpu_id": gid, "self_pid": os.getpid(), "self_in_kfd": os.getpid() in kfd_pids()}
    print(res, flush=True)
    for kind in ("idle", "spin", "duty", "resnet"):
        p = start(kind, a.secs + 3)
        time.sleep(0.5)
        res[kind] = sample([p.hostpid], gid, a.secs)
        p.wait(60)
        print(kind, json.dumps(res[kind]), flush=True)
    ps = [start("spin", a.secs + 3), start("spin", a.secs + 3)]
    res["two_spin_hostpids"] = [p.hostpid for p in ps]
    time.sleep(0.5)
    res["two_spin"] = sample([p.hostpid for p in ps], gid, a.secs)
    for p in ps:
        p.wait(60)
    print("two_spin", json.dumps(res["two_spin"]), flush=True)
    res["shim_hostpid"] = shim_hostpids(4)
    print("shim_hostpid", json.dumps(res["shim_hostpid"]), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(res, open(a.out, "w"), indent=1)


def shim_hostpids(n):
    """n GPU processes of one vGPU container started together: which host PIDs did the
    shim record in the region?"""
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    from amdvgpu.shim.region import Region
    c = vgpu_env(mem_limit=8 << 30)
    code = "import torch,time; torch.zeros(1,device='cuda'); torch.cuda.synchronize(); print('READY',flush=True); time.sleep(3)"
    ps = [subprocess.Popen([sys.executable, "-c", code], env=apply_contract(c), stdout=subprocess.PIPE, text=True)
          for _ in range(n)]
    try:
        for p in ps:
            p.stdout.readline()
        kfd = sorted(kfd_pids())
        with Region(c["VGPU_SHARED_CACHE"]) as r:
            procs = r.procs()
        return {"procs": [{k: v for k, v in pr.items() if k in ("pid", "hostpid")} for pr in procs],
                "children": [p.pid for p in ps], "kfd": kfd}
    finally:
        for p in ps:
            p.wait(30)
        cleanup_region(c)


if __name__ == "__main__":
    main()
