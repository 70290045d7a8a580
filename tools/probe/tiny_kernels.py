#!/usr/bin/env python3
"""How fast does one MI355X run tiny kernels from N processes at once? Each process launches
`spin(nblocks, us)` back to back (a synchronize every 64 launches) for a fixed window and
reports kernels/s. Process i runs on the CPUs of NUMA node i mod n (one socket each, two
per socket from 3 processes on), so the per-socket effect of profiles/r5d is held constant.
Kernels of this size need no host work beyond the launch, so the numbers separate the GPU's
handling of several processes' queues from PyTorch's host path (profiles/r5k).

    python tools/probe/tiny_kernels.py --procs 1,2,3,4,8 --nblocks 8 --us 5 --seconds 3
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


def node_cpus():
    allowed = os.sched_getaffinity(0)
    out = []
    for d in sorted(glob.glob("/sys/devices/system/node/node[0-9]*")):
        cpus = set()
        for part in open(os.path.join(d, "cpulist")).read().strip().split(","):
            lo, _, hi = part.partition("-")
            if lo:
                cpus.update(range(int(lo), int(hi or lo) + 1))
        if cpus & allowed:
            out.append(sorted(cpus & allowed))
    return out or [sorted(allowed)]


def tenant(a):
    if a.cpus:
        os.sched_setaffinity(0, {int(c) for c in a.cpus.split(",")})
    import torch
    from amdvgpu.ops import spin
    spin(a.nblocks, a.us)
    torch.cuda.synchronize()
    open(a.go + f".ready.{os.getpid()}", "w").close()
    while not os.path.exists(a.go):
        time.sleep(0.001)
    if a.wait == "block":
        def sync():
            ev = torch.cuda.Event(blocking=True)
            ev.record()
            ev.synchronize()
    else:
        sync = torch.cuda.synchronize
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < a.seconds:
        spin(a.nblocks, a.us)
        n += 1
        if n % a.sync_every == 0:
            sync()
    torch.cuda.synchronize()
    print(json.dumps({"kernels_per_s": round(n / (time.perf_counter() - t0), 1)}), flush=True)


def point(a, procs):
    go = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"tiny-go-{os.getpid()}-{procs}")
    nodes = node_cpus()
    ps = []
    env = dict(os.environ)
    if a.shim:   # each process a quota-only vGPU of its own (the shim preloaded, no limits)
        from amdvgpu.shim.launcher import apply_contract, vgpu_env
    for i in range(procs):
        if a.shim:
            env = apply_contract(vgpu_env(mem_limit=64 << 30, cu_limit=a.cu_limit or None))
        env.update(dict(kv.split("=", 1) for kv in a.env))
        cpus = nodes[i % len(nodes)][(i // len(nodes)) * 4:(i // len(nodes)) * 4 + 4]
        ps.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--tenant", "--go", go,
                                    "--nblocks", str(a.nblocks), "--us", str(a.us), "--seconds", str(a.seconds),
                                    "--cpus", ",".join(map(str, cpus)), "--wait", a.wait,
                                    "--sync-every", str(a.sync_every)], stdout=subprocess.PIPE, text=True, env=env))
    t_end = time.time() + 300
    while len(glob.glob(go + ".ready.*")) < procs and time.time() < t_end:
        if any(p.poll() not in (None, 0) for p in ps):
            break
        time.sleep(0.05)
    open(go, "w").close()
    rates = [json.loads(p.communicate(timeout=300)[0].strip().splitlines()[-1])["kernels_per_s"] for p in ps]
    for f in glob.glob(go + "*"):
        os.unlink(f)
    return rates


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", default="1,2,3,4,8")
    ap.add_argument("--nblocks", type=int, default=8)
    ap.add_argument("--us", type=int, default=5)
    ap.add_argument("--seconds", type=float, default=3.0)
    ap.add_argument("--tenant", action="store_true")
    ap.add_argument("--go")
    ap.add_argument("--cpus", default="")
    ap.add_argument("--wait", default="spin", choices=["spin", "block"],
                    help="torch.cuda.synchronize (HIP spins) or a blocking event wait")
    ap.add_argument("--sync-every", type=int, default=64)
    ap.add_argument("--shim", action="store_true", help="run every process in a quota-only vGPU")
    ap.add_argument("--cu-limit", type=int, default=0, help="with --shim: the vGPUs' CU share (auto mode)")
    ap.add_argument("--env", action="append", default=[], help="KEY=VALUE for every process")
    a = ap.parse_args()
    if a.tenant:
        return tenant(a)
    one = None
    for n in [int(x) for x in a.procs.split(",")]:
        rates = point(a, n)
        agg = sum(rates)
        one = one or agg
        print(json.dumps({"procs": n, "nblocks": a.nblocks, "us": a.us, "wait": a.wait, "sync_every": a.sync_every,
                          "shim": a.shim, "cu_limit": a.cu_limit, "env": a.env, "aggregate_kernels_per_s": round(agg, 1),
                          "vs_one": round(agg / one, 3), "per_proc": rates}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
