#!/usr/bin/env python3
"""Side-by-side fused-MFMA time (us) and TFLOP/s per layer of several
benchmarks/conv_bench.py markdown tables.

    python tools/conv_compare.py profiles/r1ag/conv.md gpurun_out/r1aj/conv.md ...
"""
import sys


def read(path):
    rows, hdr = {}, None
    for line in open(path):
        c = [x.strip() for x in line.split("|")][1:-1]
        if not c or c[0].startswith("---"):
            continue
        if c[0] in ("layer", "block"):
            hdr = c
            continue
        rows[c[0]] = dict(zip(hdr, c))
    return rows


def main(paths):
    tabs = [read(p) for p in paths]
    print("| layer | " + " | ".join(f"us ({p.split('/')[-2]})" for p in paths) + " | "
          + " | ".join(f"TF ({p.split('/')[-2]})" for p in paths) + " |")
    print("|---" * (1 + 2 * len(paths)) + "|")
    for k in tabs[0]:
        us = [t.get(k, {}).get("fused MFMA us", t.get(k, {}).get("dual us", "-")) for t in tabs]
        tf = [t.get(k, {}).get("fused TFLOP/s", t.get(k, {}).get("dual TFLOP/s", "")) for t in tabs]
        print(f"| {k} | " + " | ".join(us) + " | " + " | ".join(tf) + " |")


if __name__ == "__main__":
    main(sys.argv[1:])
