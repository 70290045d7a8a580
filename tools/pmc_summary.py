#!/usr/bin/env python3
"""Summarise rocprofv3 ``--pmc`` counter CSVs (``*_counter_collection.csv``) per kernel
family, one column group per run, as markdown.

    python tools/pmc_summary.py native=OUT/a/native_counter_collection.csv \\
        vgpu50=OUT/b/v50_counter_collection.csv ... [--title T] [-o out.md]

For every (run, kernel family) it reports dispatches, mean ``SIMD_UTILIZATION`` (busy
CU-cycles / (cycles x CUs): the fraction of the chip's CUs a dispatch kept busy) and the
raw SQ_WAVES / SQ_BUSY_CU_CYCLES / GRBM_GUI_ACTIVE sums, plus mean dispatch duration
when the CSV has timestamps.
"""
import argparse
import collections
import csv
import glob
import re

FAMILIES = [
    ("spin (vgpu_spin, 8 WG/CU)", r"spin_kernel"),
    ("CK / MIOpen convolution", r"conv_fwd|igemm|naive_conv|grouped_conv"),
    ("other", r"."),
]


def family(name):
    for fam, pat in FAMILIES:
        if re.search(pat, name):
            return fam
    return "other"


def load(path):
    """{dispatch_id: {"name", "dur_ns", counters...}}"""
    out = {}
    with open(path, newline="") as f:
        for row in csv.DictReader(f):
            did = row.get("Dispatch_Id") or row.get("Correlation_Id")
            d = out.setdefault(did, {"name": row.get("Kernel_Name", "?")})
            try:
                d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])
            except (KeyError, ValueError):
                pass
            s, e = row.get("Start_Timestamp"), row.get("End_Timestamp")
            if s and e and s.isdigit() and e.isdigit():
                d["dur_ns"] = int(e) - int(s)
    return out


def summarize(runs, title):
    counters = ["SIMD_UTILIZATION", "SQ_WAVES", "SQ_BUSY_CU_CYCLES", "GRBM_GUI_ACTIVE"]
    lines = [f"# {title}", "", "| run | kernel family | dispatches | mean SIMD_UTILIZATION | max SIMD_UTILIZATION "
             "| SQ_WAVES (sum) | SQ_BUSY_CU_CYCLES (sum) | GRBM_GUI_ACTIVE (sum) | mean dispatch us |",
             "|---|---|---|---|---|---|---|---|---|"]
    for label, path in runs:
        data = load(path)
        fams = collections.defaultdict(list)
        for d in data.values():
            fams[family(d["name"])].append(d)
        for fam, _ in FAMILIES:
            ds = fams.get(fam)
            if not ds:
                continue
            util = [d["SIMD_UTILIZATION"] for d in ds if "SIMD_UTILIZATION" in d]
            sums = {c: sum(d.get(c, 0.0) for d in ds) for c in counters[1:]}
            durs = [d["dur_ns"] for d in ds if "dur_ns" in d]
            lines.append(
                f"| {label} | {fam} | {len(ds)} | {sum(util) / len(util):.3f} | {max(util):.3f} | "
                f"{sums['SQ_WAVES']:.4g} | {sums['SQ_BUSY_CU_CYCLES']:.4g} | {sums['GRBM_GUI_ACTIVE']:.4g} | "
                f"{(sum(durs) / len(durs) / 1e3) if durs else float('nan'):.1f} |"
                if util else f"| {label} | {fam} | {len(ds)} | - | - | - | - | - | - |")
    return "\n".join(lines) + "\n"


def summarize_all(runs, title):
    """One row per (run, kernel name): dispatches, mean duration and the per-dispatch mean
    of every counter present."""
    lines = [f"# {title}", ""]
    for label, path in runs:
        data = load(path)
        names = sorted({c for d in data.values() for c in d if c not in ("name", "dur_ns")})
        by = collections.defaultdict(list)
        for d in data.values():
            by[d["name"]].append(d)
        lines += [f"## {label}", "", "| kernel | dispatches | mean us | " + " | ".join(names) + " |",
                  "|---|---|---|" + "---|" * len(names)]
        for kname, ds in sorted(by.items(), key=lambda kv: -sum(d.get("dur_ns", 0) for d in kv[1])):
            durs = [d["dur_ns"] for d in ds if "dur_ns" in d]
            short = (kname if len(kname) < 70 else kname[:67] + "...").replace("|", "\\|")
            vals = [sum(d.get(c, 0.0) for d in ds) / len(ds) for c in names]
            lines.append(f"| `{short}` | {len(ds)} | {(sum(durs) / len(durs) / 1e3) if durs else float('nan'):.1f} | "
                         + " | ".join(f"{v:.4g}" for v in vals) + " |")
        lines.append("")
    return "\n".join(lines) + "\n"


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("runs", nargs="+", help="label=path (path may be a glob)")
    ap.add_argument("--title", default="rocprofv3 --pmc summary")
    ap.add_argument("--all-counters", action="store_true", help="per-kernel table of every counter in the CSVs")
    ap.add_argument("-o", "--out")
    a = ap.parse_args()
    runs = []
    for r in a.runs:
        label, _, pat = r.partition("=")
        paths = sorted(glob.glob(pat, recursive=True))
        if not paths:
            raise SystemExit(f"no file matches {pat}")
        runs += [(label, p) for p in paths]
    text = summarize_all(runs, a.title) if a.all_counters else summarize(runs, a.title)
    if a.out:
        open(a.out, "w").write(text)
    print(text)


if __name__ == "__main__":
    main()
