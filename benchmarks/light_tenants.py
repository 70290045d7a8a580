#!/usr/bin/env python3
"""Light tenants under the GPU-time limiter: where does a co-running tenant's shortfall
come from?

A light tenant (stock fp32 ResNet-50 inference at batch 4: launch-bound, the GPU idles
between its kernels) at a 25 % GPU-time limit gets ~33-35 % of its native throughput
alone (25 % of the GPU's time is a third of its work when it keeps the GPU only ~75 %
busy by itself). Four such tenants at once got 28-31 % each in round 3, sometimes ~33 %.
This study separates the causes in one window, each arm with fresh processes:

    native x1            the reference throughput (no shim)
    native x4            four unmanaged tenants: what the GPU and the host give four
    unlimited x4         four vGPUs without a compute limit (shim cost under contention)
    limited x1 / x4      25 % temporal, alone and together
    (--ab-shim PATH)     the last two arms again with another build of the shim

Per tenant it reports the throughput as a percentage of native, the container's charged
share of the GPU's time and the fraction of the run its launches spent blocked at the
gate (throttle). If the limited tenants are charged < 25 % and hardly throttled, the
limiter is not what holds them back: four launch-bound processes share the GPU's
instants and the host, and `unlimited x4 / 4` is their ceiling.

    python benchmarks/light_tenants.py [--seconds 5] [--repeats 2] [--ab-shim lib.so]
"""
import argparse
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "benchmarks"))

from temporal_accuracy import run_tenants  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=5.0)
    ap.add_argument("--batch", type=int, default=4)
    ap.add_argument("--limit", type=int, default=25)
    ap.add_argument("--tenants", type=int, default=4)
    ap.add_argument("--repeats", type=int, default=1)
    ap.add_argument("--ab-shim", default="", help="another libvgpu_hip.so for the limited arms (A/B)")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    from amdvgpu.shim.launcher import vgpu_env
    n = a.tenants
    GiB = 1 << 30

    def limited():
        return vgpu_env(cu_limit=a.limit, cu_mode="temporal", mem_limit=32 * GiB)

    arms = [("native x1", lambda: [None], None), (f"native x{n}", lambda: [None] * n, None),
            (f"unlimited x{n}", lambda: [vgpu_env(mem_limit=32 * GiB) for _ in range(n)], None),
            (f"limited {a.limit}% x1", lambda: [limited()], None),
            (f"limited {a.limit}% x{n}", lambda: [limited() for _ in range(n)], None)]
    if a.ab_shim:
        tag = os.path.basename(a.ab_shim)
        arms += [(f"limited {a.limit}% x1 [{tag}]", lambda: [limited()], a.ab_shim),
                 (f"limited {a.limit}% x{n} [{tag}]", lambda: [limited() for _ in range(n)], a.ab_shim),
                 (f"unlimited x{n} [{tag}]", lambda: [vgpu_env(mem_limit=32 * GiB) for _ in range(n)], a.ab_shim)]
    rows = []
    for rep in range(a.repeats):
        native = None
        for name, make, shim in arms:
            res = run_tenants("resnet50", make(), a.seconds, 8, a.batch, shim=shim, full=True)
            if name == "native x1":
                native = res[0]["throughput"]
            row = {"repeat": rep, "arm": name, "native": native,
                   "pct": [100.0 * r["throughput"] / native for r in res],
                   "charged_pct": [r.get("charged_pct") for r in res],
                   "throttle_pct": [r.get("throttle_pct") for r in res]}
            row["aggregate_pct"] = sum(row["pct"])
            rows.append(row)
            print(json.dumps(row), flush=True)

    def fmt(xs):
        return " / ".join("-" if x is None else f"{x:.1f}" for x in xs)

    md = [f"# light tenants — ResNet-50 b={a.batch} fp32, {a.seconds:.0f} s per arm", "",
          "| rep | arm | % of native (each) | aggregate % | charged % of GPU time | throttled % of run |",
          "|---|---|---|---|---|---|"]
    for r in rows:
        md.append(f"| {r['repeat']} | {r['arm']} | {fmt(r['pct'])} | {r['aggregate_pct']:.1f} | "
                  f"{fmt(r['charged_pct'])} | {fmt(r['throttle_pct'])} |")
    print("\n".join(md))
    if a.json_out:
        json.dump(rows, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
