#!/usr/bin/env python3
"""Where a GPU-bound pod's CPU time goes: stock fp32 ResNet-50 b=50 inference for a fixed
wall time (a blocking wait every 4 steps, as bench.py's concurrent pods), natively and in a
quota-only vGPU, with every thread's CPU seconds in the window (by TID and name).

    python tools/probe/cpu_probe.py [--seconds 6] [--modes native,vgpu] [--sync block|spin|every]
"""
import argparse
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def thread_cpu():
    tick = os.sysconf("SC_CLK_TCK")
    out = {}
    for t in os.listdir("/proc/self/task"):
        try:
            st = open(f"/proc/self/task/{t}/stat").read()
            name = st[st.index("(") + 1:st.rindex(")")]
            f = st[st.rindex(")") + 2:].split()
            out[int(t)] = (name, (int(f[11]) + int(f[12])) / tick)
        except (OSError, ValueError, IndexError):
            pass
    return out


def tenant(seconds, sync_mode, case):
    import resource

    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = True
    r = Runner(get_case(case), "cuda:0", dtype=torch.float32)
    for _ in range(5):
        r.step()
    torch.cuda.synchronize()

    def wait():
        if sync_mode == "spin":
            torch.cuda.synchronize()
        else:
            ev = torch.cuda.Event(blocking=True)
            ev.record()
            ev.synchronize()

    every = 1 if sync_mode == "every" else 4
    c0, ru0 = thread_cpu(), resource.getrusage(resource.RUSAGE_SELF)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r.step()
        n += 1
        if n % every == 0:
            wait()
    wait()
    dt = time.perf_counter() - t0
    c1, ru1 = thread_cpu(), resource.getrusage(resource.RUSAGE_SELF)
    per = []
    for tid, (name, cpu) in c1.items():
        d = cpu - c0.get(tid, (name, 0.0))[1]
        if d >= 0.01:
            per.append({"tid": tid, "main": tid == os.getpid(), "name": name, "cpu_s": round(d, 2)})
    per.sort(key=lambda x: -x["cpu_s"])
    print(json.dumps({"ms_per_step": round(dt * 1000 / n, 3), "window_s": round(dt, 2),
                      "cpus_busy": round((ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime) / dt, 3),
                      "vol_ctx": ru1.ru_nvcsw - ru0.ru_nvcsw, "threads": per}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--modes", default="native,vgpu")
    ap.add_argument("--sync", default="block", choices=["block", "spin", "every"])
    ap.add_argument("--case", default="resnet50-inf")
    ap.add_argument("--tenant", action="store_true")
    ap.add_argument("--extra-env", action="append", default=[], help="KEY=VALUE for every mode")
    a = ap.parse_args()
    if a.tenant:
        return tenant(a.seconds, a.sync, a.case)
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    for mode in a.modes.split(","):
        c = vgpu_env(mem_limit=64 << 30) if mode == "vgpu" else None
        env = apply_contract(c) if c else dict(os.environ)
        env.update(dict(kv.split("=", 1) for kv in a.extra_env))
        try:
            out = subprocess.run([sys.executable, os.path.abspath(__file__), "--tenant", "--seconds", str(a.seconds),
                                  "--sync", a.sync, "--case", a.case], env=env, capture_output=True, text=True,
                                 timeout=300)
        finally:
            if c:
                cleanup_region(c)
        line = [l for l in out.stdout.splitlines() if l.startswith("{")]
        print(mode, a.sync, " ".join(a.extra_env), line[-1] if line else out.stderr[-2000:], flush=True)
        for l in out.stderr.splitlines():   # VGPU_STATS=1: the shim's per-process counters
            if l.startswith("[vGPU stats"):
                print("   ", l, flush=True)
        if out.returncode != 0:
            raise SystemExit(out.returncode)


if __name__ == "__main__":
    main()
