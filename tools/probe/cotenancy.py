#!/usr/bin/env python3
"""Do two launch-bound processes' kernels ever run at the same time on one MI355X?

Round 4 measured two unmasked LSTM inference processes at 1.00x aggregate (profiles/r4h)
where round 2 had 1.78x, and asserted "the box" without evidence. This probe runs N stock
PyTorch tenants of one case side by side (no shim, no mask), each timing its own steps, for
a rocprofv3 kernel trace of all of them; --analyze then reads the per-process kernel traces
and reports, over the window in which all of them run:

    busy        fraction of the window each process has a kernel executing
    both        fraction in which kernels of every process execute at once (true overlap)
    any         fraction in which some kernel executes (the GPU's busy time)
    gap_us      each process's gaps between consecutive kernels (median / p90 / p99): how
                long its queue stays empty while the other one runs
    long_gap_share  the share of the window each process spends in gaps of >= 100 us

If `both` stays ~0 while each process's gaps are as long as the other's bursts, the GPU
time-slices the processes' queues (the hardware scheduler switching between process
contexts) rather than running their kernels concurrently.

    python3 tools/probe/cotenancy.py --case lstm-inf --procs 2 --seconds 4 --trace OUT
    python3 tools/probe/cotenancy.py --analyze OUT

--trace runs every tenant under its own rocprofv3 (--kernel-trace, csv, OUT/t<i>): the
launcher itself never loads the GPU runtime, and each tenant's trace lands in a directory of
its own (rocprofv3's timestamps share one clock across the processes of a host).
"""
import argparse
import csv
import glob
import json
import os
import subprocess
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, REPO)


def tenant(case, seconds, go, batch):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = True
    r = Runner(get_case(case), "cuda:0", dtype=torch.float32, batch=batch or None)
    for _ in range(5):
        r.step()
    torch.cuda.synchronize()
    open(go + f".ready.{os.getpid()}", "w").close()
    while not os.path.exists(go):
        time.sleep(0.001)
    n, t0 = 0, time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r.step()
        n += 1
        if n % 4 == 0:
            torch.cuda.synchronize()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    print(json.dumps({"pid": os.getpid(), "case": case, "steps": n, "ms_per_step": round(dt * 1e3 / n, 3),
                      "items_per_s": round(n * r.items_per_step / dt, 1)}), flush=True)


def launch(a):
    go = os.path.join(os.environ.get("TMPDIR", "/tmp"), f"cotenancy-go-{os.getpid()}")
    args = [sys.executable, os.path.abspath(__file__), "--tenant", "--case", a.case, "--seconds", str(a.seconds),
            "--go", go] + (["--batch", str(a.batch)] if a.batch else [])
    def cmd(i):
        if not a.trace:
            return args
        return ["rocprofv3", "--kernel-trace", "--output-format", "csv", "-d", os.path.join(a.trace, f"t{i}"),
                "-o", f"t{i}", "--"] + args
    procs = [subprocess.Popen(cmd(i), stdout=subprocess.PIPE, text=True) for i in range(a.procs)]
    deadline = time.time() + 600
    while len(glob.glob(go + ".ready.*")) < a.procs and time.time() < deadline:
        if any(p.poll() not in (None, 0) for p in procs):
            break
        time.sleep(0.05)
    open(go, "w").close()
    def result(p):   # the tenant's line (rocprofv3 prints its own lines around it)
        lines = [ln for ln in p.communicate(timeout=600)[0].splitlines() if ln.startswith('{"pid"')]
        return json.loads(lines[-1])
    outs = [result(p) for p in procs]
    for f in glob.glob(go + "*"):
        os.unlink(f)
    agg = sum(o["items_per_s"] for o in outs)
    print(json.dumps({"case": a.case, "procs": a.procs, "aggregate_items_per_s": round(agg, 1), "tenants": outs}),
          flush=True)
    return 0 if all(p.returncode == 0 for p in procs) else 1


def merge(iv):
    out = []
    for s, e in sorted(iv):
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def clip(iv, lo, hi):
    return [[max(s, lo), min(e, hi)] for s, e in iv if e > lo and s < hi]


def length(iv):
    return sum(e - s for s, e in iv)


def intersect(a, b):
    out, i, j = [], 0, 0
    while i < len(a) and j < len(b):
        s, e = max(a[i][0], b[j][0]), min(a[i][1], b[j][1])
        if s < e:
            out.append([s, e])
        if a[i][1] < b[j][1]:
            i += 1
        else:
            j += 1
    return out


def pct(xs, q):
    xs = sorted(xs)
    return xs[min(len(xs) - 1, int(q * len(xs)))] if xs else 0


def _tenant_of_path(d, f):
    # --trace puts tenant i's files under d/t<i>/...
    return os.path.relpath(f, d).split(os.sep)[0]


def analyze(d):
    per = {}
    for f in glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                pid = _tenant_of_path(d, f)
                try:
                    s, e = int(row["Start_Timestamp"]), int(row["End_Timestamp"])
                except (KeyError, ValueError):
                    continue
                per.setdefault(str(pid), []).append((s, e))
    # tenants only: the launcher itself runs no kernels
    per = {p: merge(iv) for p, iv in per.items() if len(iv) > 100}
    if not per:
        return {"error": f"no kernel traces under {d}"}
    lo = max(iv[0][0] for iv in per.values())
    hi = min(iv[-1][1] for iv in per.values())
    span = hi - lo
    lo, hi = lo + span // 10, hi - span // 10   # the steady middle of the common window
    win = hi - lo
    res = {"window_ms": round(win / 1e6, 1), "procs": {}}
    clipped = {p: clip(iv, lo, hi) for p, iv in per.items()}
    both = None
    for p, iv in clipped.items():
        gaps = [b[0] - a[1] for a, b in zip(iv, iv[1:])]
        res["procs"][p] = {"busy": round(length(iv) / win, 4), "kernels": len(iv),
                           "gap_us_median": round(pct(gaps, 0.5) / 1e3, 1), "gap_us_p90": round(pct(gaps, 0.9) / 1e3, 1),
                           "gap_us_p99": round(pct(gaps, 0.99) / 1e3, 1),
                           # idle time in gaps of 100 us or more (where another queue could run)
                           "long_gap_share": round(sum(g for g in gaps if g >= 100_000) / win, 4),
                           "kernel_us_median": round(pct([e - s for s, e in iv], 0.5) / 1e3, 1)}
        both = iv if both is None else intersect(both, iv)
    res["both"] = round(length(both) / win, 4) if len(clipped) > 1 else None
    res["any"] = round(length(merge([x for iv in clipped.values() for x in iv])) / win, 4)
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="lstm-inf")
    ap.add_argument("--procs", type=int, default=2)
    ap.add_argument("--seconds", type=float, default=4.0)
    ap.add_argument("--batch", type=int, default=0)
    ap.add_argument("--tenant", action="store_true")
    ap.add_argument("--go")
    ap.add_argument("--analyze")
    ap.add_argument("--trace", default="", help="rocprofv3 kernel trace of every tenant under this directory")
    a = ap.parse_args()
    if a.analyze:
        print(json.dumps(analyze(a.analyze)))
        return 0
    if a.tenant:
        return tenant(a.case, a.seconds, a.go, a.batch)
    return launch(a)


if __name__ == "__main__":
    sys.exit(main())
