#!/usr/bin/env python3
"""rocprofv3 evidence for the data plane: the same stock fp32 ResNet-50 tenant profiled
natively, inside a quota-only vGPU, and inside a 25 % temporal vGPU with the shim's roctx
ranges on (VGPU_TRACE=1).

    python tools/probe/prof_tenant.py --out gpurun_out/prof [--steps 30] [--case resnet50-inf]
        [--modes native,vgpu-quota,vgpu-t25] [--runs 1] [--autotune 1]

For every mode (and run): `rocprofv3 --kernel-trace --marker-trace --stats -d
<out>/<mode>.<run> -- python3 prof_tenant.py --tenant ...` (the profiled program itself
follows `--`), then a summary (wall and GPU kernel time per step, top kernels, vgpu:*
marker time) in <out>/summary.md. With --runs > 1 the same mode is profiled in several
processes, which separates process-to-process variation (e.g. MIOpen picking different
convolution solvers under autotuning) from the cost of the interception.
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


def tenant(steps, case, autotune):
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = bool(autotune)
    r = Runner(get_case(case), "cuda:0", dtype=torch.float32)
    for _ in range(5):
        r.step()
    torch.cuda.synchronize()
    # The timed window as a roctx range: the summary counts only the kernels inside it
    # (warm-up, MIOpen find and model loading stay out of the per-step figures).
    # rocprofv3 records the rocprofiler-sdk roctx (as the shim's own ranges use, trace.cpp);
    # the legacy libroctx64 is only the fallback.
    import ctypes
    roctx = None
    for lib in ("librocprofiler-sdk-roctx.so.1", "/opt/rocm/lib/librocprofiler-sdk-roctx.so.1", "libroctx64.so.4"):
        try:
            roctx = ctypes.CDLL(lib, mode=ctypes.RTLD_GLOBAL)
            break
        except OSError:
            continue
    if roctx:
        roctx.roctxRangePushA(b"vgpu-prof:timed")
    t0 = time.perf_counter()
    for _ in range(steps):
        r.step()
    torch.cuda.synchronize()
    if roctx:
        roctx.roctxRangePop()
    print(json.dumps({"ms_per_step": (time.perf_counter() - t0) * 1000 / steps}), flush=True)


def find(d, pattern):
    hits = glob.glob(os.path.join(d, "**", pattern), recursive=True)
    return hits[0] if hits else None


def _union_ms(intervals):
    total, cur_s, cur_e = 0.0, None, None
    for s, e in sorted(intervals):
        if cur_e is None or s > cur_e:
            if cur_e is not None:
                total += cur_e - cur_s
            cur_s, cur_e = s, e
        else:
            cur_e = max(cur_e, e)
    if cur_e is not None:
        total += cur_e - cur_s
    return total / 1e6


def timed_window(d, steps):
    """Steady-state figures from the kernel trace, restricted to the tenant's timed window
    (roctx range vgpu-prof:timed): GPU busy time per step (union of kernel intervals), the
    busy fraction of the window, kernels per step and the top kernels inside it."""
    kt, mk = find(d, "*kernel_trace.csv"), find(d, "*marker_api_trace.csv")
    if not kt or not mk:
        return {}
    win = None
    for r in csv.DictReader(open(mk)):
        if (r.get("Function") or r.get("Name") or "") == "vgpu-prof:timed":
            win = (float(r["Start_Timestamp"]), float(r["End_Timestamp"]))
    if not win:
        return {}
    t0, t1 = win
    ivs, per = [], {}
    for r in csv.DictReader(open(kt)):
        s, e = float(r["Start_Timestamp"]), float(r["End_Timestamp"])
        if e <= t0 or s >= t1:
            continue
        s, e = max(s, t0), min(e, t1)
        ivs.append((s, e))
        name = r.get("Kernel_Name") or r.get("Name") or "?"
        per[name] = per.get(name, 0.0) + (e - s)
    busy = _union_ms(ivs)
    wall = (t1 - t0) / 1e6
    top = sorted(per.items(), key=lambda kv: -kv[1])[:5]
    return {"window_ms": round(wall, 2), "busy_ms_per_step": round(busy / steps, 3),
            "busy_fraction": round(busy / wall, 4) if wall else None, "kernels_per_step": round(len(ivs) / steps, 1),
            "top_timed": [(n[:70], round(t / 1e6 / steps, 3)) for n, t in top]}


def hip_api_table(out, keys):
    """Per-function HIP API call counts and mean duration (whole process) for every mode,
    from rocprofv3's hip_api_stats.csv, the functions with the most total time first."""
    per = {}
    for k in keys:
        f = find(os.path.join(out, k), "*hip_api_stats.csv")
        for r in (csv.DictReader(open(f)) if f else []):
            per.setdefault(r["Name"], {})[k] = (int(r["Calls"]), float(r["TotalDurationNs"]))
    names = sorted(per, key=lambda n: -max(t for _, t in per[n].values()))[:25]
    md = ["| HIP function | " + " | ".join(f"{k} calls / mean us" for k in keys) + " |", "|---|" + "---|" * len(keys)]
    for n in names:
        cells = []
        for k in keys:
            c, t = per[n].get(k, (0, 0.0))
            cells.append(f"{c} / {t / c / 1e3:.2f}" if c else "-")
        md.append(f"| {n} | " + " | ".join(cells) + " |")
    return "\n".join(md)


def summarize(d, steps):
    out = timed_window(d, steps)
    ks = find(d, "*kernel_stats.csv")
    if ks:
        rows = list(csv.DictReader(open(ks)))
        total = sum(float(r["TotalDurationNs"]) for r in rows)
        out["kernel_ms_per_step"] = total / 1e6 / (steps + 5)
        out["kernels"] = sum(int(r["Calls"]) for r in rows)
        top = sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5]
        out["top"] = [(r["Name"][:70], round(float(r["TotalDurationNs"]) / 1e6, 2), int(r["Calls"])) for r in top]
        out["kernel_names"] = len(rows)
    mk = find(d, "*marker_api_trace.csv")
    if mk:
        rows = list(csv.DictReader(open(mk)))
        agg = {}
        for r in rows:
            name = r.get("Function") or r.get("Name") or ""
            if name.startswith("vgpu:"):
                dur = float(r["End_Timestamp"]) - float(r["Start_Timestamp"])
                n, t = agg.get(name, (0, 0.0))
                agg[name] = (n + 1, t + dur / 1e6)
        out["markers"] = {k: {"count": n, "ms": round(t, 2)} for k, (n, t) in agg.items()}
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--out", default="gpurun_out/prof")
    ap.add_argument("--steps", type=int, default=30)
    ap.add_argument("--tenant", action="store_true")
    ap.add_argument("--case", default="resnet50-inf")
    ap.add_argument("--modes", default="native,vgpu-quota,vgpu-t25")
    ap.add_argument("--runs", type=int, default=1)
    ap.add_argument("--autotune", type=int, default=1)
    ap.add_argument("--hip-api", action="store_true", help="also trace the HIP runtime API (per-function call "
                    "counts and time in <out>/hip_api.md)")
    ap.add_argument("--prewarm", type=int, default=1, help="run the tenant once unprofiled first (fills MIOpen's "
                    "find-db, so no profiled process pays the search)")
    a = ap.parse_args()
    if a.tenant:
        return tenant(a.steps, a.case, a.autotune)
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    pods = {}

    def pod_env(ledger):
        # the suite's interception-only pod (benchmarks/aibench_suite.py: split 2, cores
        # scaling 2, memory scaling 1.8), through a plugin and stub kubelet
        if ledger not in pods:
            from amdvgpu.plugin.devices import SysfsBackend
            from amdvgpu.plugin.kubelet_stub import NodeHarness
            backend = SysfsBackend()
            h = NodeHarness(backend, device_split_count=2, device_memory_scaling=1.8, host_memory_fraction=0.0,
                            device_cores_scaling=2.0, ledger=ledger)
            h.__enter__()
            pods[ledger] = (h, backend.devices()[0].uuid)
        h, uuid = pods[ledger]
        envs, mounts = h.pod(h.vgpu_ids(uuid)[:1])
        return apply_contract(envs, mounts)

    contracts = {
        "native": lambda: None,
        "vgpu-pod": lambda: "pod",
        "vgpu-pod-noledger": lambda: "pod-noledger",
        "vgpu-quota": lambda: vgpu_env(mem_limit=72 << 30),
        "vgpu-t25": lambda: vgpu_env(mem_limit=72 << 30, cu_limit=25, cu_mode="temporal", extra={"VGPU_TRACE": "1"}),
    }
    res = {}
    if a.prewarm:
        subprocess.run([sys.executable, os.path.abspath(__file__), "--tenant", "--steps", "3", "--case", a.case,
                        "--autotune", str(a.autotune)], check=True, timeout=600)
    for run in range(a.runs):
        for mode in (a.modes.split(",") if run % 2 == 0 else a.modes.split(",")[::-1]):
            c = contracts[mode]()
            if isinstance(c, str):
                env, c = pod_env(c == "pod"), None
            else:
                env = apply_contract(c) if c else dict(os.environ)
            key = mode if a.runs == 1 else f"{mode}.{run}"
            d = os.path.join(a.out, key)
            cmd = ["rocprofv3", "--kernel-trace", "--marker-trace", *(["--hip-runtime-trace"] if a.hip_api else []),
                   "--stats", "--output-format", "csv", "-d", d, "-o", mode, "--",
                   sys.executable, os.path.abspath(__file__), "--tenant", "--steps", str(a.steps), "--case", a.case,
                   "--autotune", str(a.autotune)]
            p = subprocess.run(cmd, env=env, capture_output=True, text=True, timeout=600)
            if c:
                cleanup_region(c)
            line = [l for l in p.stdout.splitlines() if l.startswith("{")]
            res[key] = {"rc": p.returncode, **(json.loads(line[-1]) if line else {}), **summarize(d, a.steps)}
            for f in glob.glob(os.path.join(d, "**", "*"), recursive=True):  # keep the per-kernel stats only
                if os.path.isfile(f) and not f.endswith("_stats.csv"):
                    os.unlink(f)
            print(key, json.dumps(res[key]), flush=True)
            if p.returncode != 0:
                print(p.stderr[-3000:], file=sys.stderr)
                raise SystemExit(p.returncode)
    md = [f"# rocprofv3: stock fp32 {a.case} native vs inside vGPUs (autotune={a.autotune}, {a.steps} steps)", "",
          "Timed window only (roctx range `vgpu-prof:timed` around the measured steps; the find-db was "
          "filled by an unprofiled run first): GPU busy = union of kernel intervals.", "",
          "| mode | wall ms/step | GPU busy ms/step (timed) | busy fraction | kernels/step | all kernels in the process "
          "(incl. warm-up) | vgpu:* roctx ranges |",
          "|---|---|---|---|---|---|---|"]
    for m, r in sorted(res.items()):
        mk = ", ".join(f"{k} x{v['count']} {v['ms']} ms" for k, v in (r.get("markers") or {}).items()) or "-"
        md.append(f"| {m} | {r.get('ms_per_step', 0):.2f} | {r.get('busy_ms_per_step', 0):.2f} | "
                  f"{r.get('busy_fraction') or 0:.3f} | {r.get('kernels_per_step', 0)} | {r.get('kernels', 0)} | {mk} |")
    for m, r in sorted(res.items()):
        md += ["", f"Top kernels in the timed window ({m}, ms/step): " +
               "; ".join(f"{n} {t}" for n, t in r.get("top_timed", []))]
    for h, _ in pods.values():
        h.__exit__(None, None, None)
    os.makedirs(a.out, exist_ok=True)
    if a.hip_api:
        open(os.path.join(a.out, "hip_api.md"), "w").write(hip_api_table(a.out, sorted(res)) + "\n")
    open(os.path.join(a.out, "summary.md"), "w").write("\n".join(md) + "\n")
    json.dump(res, open(os.path.join(a.out, "summary.json"), "w"), indent=1)
    print("\n".join(md))


if __name__ == "__main__":
    main()
