#!/usr/bin/env python3
"""Does sampling KFD cu_occupancy at ~1 kHz slow the sampled workload down?

Runs stock fp32 ResNet-50 inference (b=50, 346²) for a fixed time three times: alone,
with this process reading the worker's cu_occupancy every 1 ms, and every 0.25 ms.
The worker's host PID is found by diffing the KFD process list around its start
(several candidates: every one of them is sampled, which only raises the cost).

    python tools/probe/sampler_overhead.py --out gpurun_out/sampler_overhead.json
"""
import argparse
import glob
import json
import os
import subprocess
import sys
import threading
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
WORKER = [sys.executable, os.path.join(REPO, "benchmarks", "temporal_accuracy.py"), "--worker", "--workload",
          "resnet50", "--sync-every", "8"]


def kfd_pids():
    return {int(d) for d in os.listdir("/sys/class/kfd/kfd/proc") if d.isdigit()}


def gpu_id():
    for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/gpu_id")):
        try:
            v = int(open(p).read().strip() or 0)
        except OSError:
            continue
        if v:
            return v
    return 0


def run(period_s, seconds, tmp):
    out = os.path.join(tmp, f"w{period_s}.json")
    go = out + ".go"
    before = kfd_pids()
    p = subprocess.Popen(WORKER + ["--seconds", str(seconds), "--out", out, "--go", go])
    while not os.path.exists(out + ".ready"):
        if p.poll() is not None:
            raise SystemExit("worker failed")
        time.sleep(0.02)
    cands = sorted(kfd_pids() - before)
    gid = gpu_id()
    paths = [f"/sys/class/kfd/kfd/proc/{c}/stats_{gid}/cu_occupancy" for c in cands]
    stop = threading.Event()
    reads = [0]

    def sampler():
        while not stop.is_set():
            for path in paths:
                try:
                    with open(path) as f:
                        f.read()
                    reads[0] += 1
                except OSError:
                    pass
            time.sleep(period_s)

    th = threading.Thread(target=sampler, daemon=True)
    if period_s:
        th.start()
    open(go, "w").close()
    p.wait(300)
    stop.set()
    res = json.load(open(out))
    res.update(period_s=period_s, candidates=len(cands), reads=reads[0])
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/sampler_overhead.json")
    ap.add_argument("--seconds", type=float, default=4.0)
    a = ap.parse_args()
    import tempfile
    tmp = tempfile.mkdtemp()
    rows = [run(p, a.seconds, tmp) for p in (0, 0.001, 0.00025, 0)]
    for r in rows:
        print(json.dumps(r), flush=True)
    os.makedirs(os.path.dirname(a.out) or ".", exist_ok=True)
    json.dump(rows, open(a.out, "w"), indent=1)


if __name__ == "__main__":
    main()
