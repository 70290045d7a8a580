#!/usr/bin/env python3
"""Diagnose the background class's yield on hardware: a priority-0 (or -2) neighbour keeps
the GPU busy with spin kernels while a background tenant (priority 2, temporal 50 %) spins;
every 50 ms the parent samples both containers' KFD occupancy (by the host PIDs in their
regions), the board slots and the background region's gate / preempt state.

    python tools/probe/bg_yield.py [--neighbour-prio 0] [--seconds 3]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests"))

GiB = 1 << 30


def occ(hostpid, gpu_id):
    try:
        return int(open(f"/sys/class/kfd/kfd/proc/{hostpid}/stats_{gpu_id}/cu_occupancy").read())
    except (OSError, ValueError):
        return -1


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--neighbour-prio", type=int, default=0)
    ap.add_argument("--seconds", type=float, default=3.0)
    a = ap.parse_args()
    from amdvgpu.shim.launcher import cleanup_region, vgpu_env
    from amdvgpu.shim.region import Region
    from conftest import child_results, spawn_child
    from test_gpu_limits import LATENCY_SPIN, SPIN_RATE
    tmp = tempfile.mkdtemp(prefix="bgy-")
    board = os.path.join(tmp, "board")
    os.makedirs(board)
    ready, stop = os.path.join(tmp, "ready"), os.path.join(tmp, "stop")
    nb = vgpu_env(mem_limit=16 * GiB, extra={"VGPU_BOARD_DIR": board, "VGPU_BOARD_SLOT": "svc.slot",
                                             "VGPU_TASK_PRIORITY": str(a.neighbour_prio)})
    bg = vgpu_env(mem_limit=16 * GiB, cu_limit=50, cu_mode="temporal",
                  extra={"VGPU_BOARD_DIR": board, "VGPU_BOARD_SLOT": "batch.slot", "VGPU_TASK_PRIORITY": "2"})
    svc = spawn_child(LATENCY_SPIN, nb, extra_env={"VGPU_TEST_READY": ready, "VGPU_TEST_GO": stop})
    samples = []
    try:
        while not os.path.exists(ready):
            if svc.poll() is not None:
                raise SystemExit("neighbour failed: " + svc.stderr.read()[-3000:])
            time.sleep(0.05)
        time.sleep(1.0)
        p = spawn_child(SPIN_RATE.format(secs=a.seconds), bg)
        t0 = time.time()
        while p.poll() is None and time.time() - t0 < a.seconds + 60:
            try:
                with Region(nb["VGPU_SHARED_CACHE"]) as rn, Region(bg["VGPU_SHARED_CACHE"]) as rb:
                    gid = rb.device(0)["gpu_id"]
                    s = {"t": round(time.time() - t0, 2),
                         "nb": [(q["hostpid"], occ(q["hostpid"], gid)) for q in rn.procs()],
                         "bg": [(q["hostpid"], occ(q["hostpid"], gid)) for q in rb.procs()],
                         "bg_dev": {k: rb.device(0)[k] for k in ("credit_ns", "preempt", "cu_mode", "charged_ns",
                                                                  "crowd", "depth_cap")},
                         "bg_samples": rb.samples, "nb_prio": rn.priority, "bg_prio": rb.priority}
            except OSError as e:
                s = {"t": round(time.time() - t0, 2), "err": str(e)}
            samples.append(s)
            time.sleep(0.05)
        o, e = p.communicate(timeout=120)
        rate = child_results(o)[0]["rate"] if p.returncode == 0 else None
        boards = sorted(os.listdir(board))
    finally:
        open(stop, "w").close()
        so, se = svc.communicate(timeout=120)
        cleanup_region(nb)
        cleanup_region(bg)
    for s in samples[:: max(1, len(samples) // 25)]:
        print(json.dumps(s, default=str))
    print(json.dumps({"rate": rate, "board": boards, "svc_rc": svc.returncode, "svc_err": se[-1500:]}, default=str))


if __name__ == "__main__":
    main()
