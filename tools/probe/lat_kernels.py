#!/usr/bin/env python3
"""Summarises the latency pod's kernel traces written by ``benchmarks/mix.py --trace-latency``.

For every traced run (``DIR/<arm>_<run>/**/*kernel_trace.csv``) the timed requests are
the last ``steps`` repetitions of the per-request kernel sequence (its period is found
from the end of the trace, so warm-up and autotuning kernels are left out). Per request:

* ``gpu_ms``   sum of the request's kernel durations (how long its kernels ran);
* ``span_ms``  first kernel start to last kernel end (kernels plus the gaps between them);
* ``gap_ms``   span - gpu: time the request's kernels waited between each other (launch,
               dispatch, queueing behind other work);
* ``first_ms`` its first kernel's duration.

Alone vs next to the trainers tells whether the service loses its time in slower kernels
(shared bandwidth / caches) or between them (dispatch). The CSVs are large; ``--prune``
deletes everything but the per-kernel stats afterwards.

    python tools/probe/lat_kernels.py DIR [--steps-json mix.json] [--prune] [--out summary.json]
"""
import argparse
import csv
import glob
import json
import os
import statistics


def period(names, max_p=4000, reps=10):
    """Smallest p whose last `reps` periods repeat the same names (the per-request kernel
    sequence; several periods, so a block repeated inside one request does not match)."""
    n = len(names)
    for p in range(1, min(max_p, n // 2) + 1):
        k = min(reps, n // p)
        if k >= 2 and all(names[n - p:] == names[n - (j + 1) * p:n - j * p] for j in range(1, k)):
            return p
    return 0


def summarize_trace(path, steps=None):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    p = period(names)
    if not p:
        return {"error": "no repeating kernel sequence", "kernels": len(rows)}
    # Requests: whole periods from the end, at most `steps` of them.
    n_req = len(rows) // p
    if steps:
        n_req = min(n_req, steps)
    # Keep only periods that repeat the final sequence exactly (autotuning differs).
    tail_names = names[len(names) - p:]
    reqs = []
    for i in range(n_req):
        lo = len(rows) - (i + 1) * p
        chunk = rows[lo:lo + p]
        if [r["Kernel_Name"] for r in chunk] != tail_names:
            break
        s = [int(r["Start_Timestamp"]) for r in chunk]
        e = [int(r["End_Timestamp"]) for r in chunk]
        gpu = sum(b - a for a, b in zip(s, e))
        span = max(e) - min(s)
        reqs.append({"gpu_ms": gpu / 1e6, "span_ms": span / 1e6, "gap_ms": (span - gpu) / 1e6,
                     "first_ms": (e[0] - s[0]) / 1e6})

    def q(key, frac):
        v = sorted(r[key] for r in reqs)
        return round(v[min(len(v) - 1, int(len(v) * frac))], 3)

    out = {"kernels_per_request": p, "requests": len(reqs)}
    for key in ("gpu_ms", "span_ms", "gap_ms"):
        out[key] = {"p50": q(key, 0.5), "p99": q(key, 0.99), "mean": round(statistics.fmean(r[key] for r in reqs), 3)}
    # Per kernel name: mean duration over the timed requests (the ten longest).
    per = {}
    for i in range(len(reqs)):
        lo = len(rows) - (i + 1) * p
        for r in rows[lo:lo + p]:
            d = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            per.setdefault(r["Kernel_Name"][:60], []).append(d)
    top = sorted(per.items(), key=lambda kv: -sum(kv[1]))[:10]
    out["top_kernels_us"] = [(k, round(statistics.fmean(v) / 1e3, 1), len(v) // max(1, len(reqs))) for k, v in top]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--steps-json", default="", help="mix.py --json-out of the same runs (request counts)")
    ap.add_argument("--prune", action="store_true")
    ap.add_argument("--out", default="")
    a = ap.parse_args()
    steps = {}
    if a.steps_json and os.path.exists(a.steps_json):
        d = json.load(open(a.steps_json))
        for r in d.get("runs", []):
            for spec, v in r.items():
                if isinstance(v, dict) and "p99_ms" in v:
                    steps[f"{r['label']}_{r['run']}"] = v
    res = {}
    for run in sorted(os.listdir(a.dir)):
        traces = glob.glob(os.path.join(a.dir, run, "**", "*kernel_trace.csv"), recursive=True)
        if not traces:
            continue
        res[run] = summarize_trace(traces[0])
        if run in steps:
            res[run]["service"] = steps[run]
        print(run, json.dumps(res[run]), flush=True)
    if a.out:
        json.dump(res, open(a.out, "w"), indent=1)
    if a.prune:
        for f in glob.glob(os.path.join(a.dir, "**", "*"), recursive=True):
            if os.path.isfile(f) and not f.endswith("_stats.csv"):
                os.unlink(f)


if __name__ == "__main__":
    main()
