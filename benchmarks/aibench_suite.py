#!/usr/bin/env python3
"""The reference's ten ai-benchmark cases on one MI355X: native, inside a vGPU, and two
concurrent vGPUs (the "virtual device memory" column), with repeat statistics.

Reference (2xV100, TF 2.4.1): native = official plugin; vGPU = this plugin
with split 2 / memScaling 1.8 (50 % SM limit + CUDA_OVERSUBSCRIBE, server.go:492,505-507);
vGPU+VDM = 4 such containers on the 2 GPUs at once ("high load", README_cn.md:52).

Every vGPU contract here comes from a real Allocate of the plugin (NodeHarness, sysfs
backend) configured like the reference's benchmark DaemonSet: --device-split-count=2
--device-memory-scaling=1.8 (default --cu-mode=auto → a 50 % spatial CU mask). The
workloads are stock PyTorch-ROCm in fp32 (MIOpen / hipBLASLt kernels, no custom ops).

Columns:
* native     no shim, the GPU visible as the official plugin would expose it
* vgpu       the pod's contract without the compute limit (the same plugin at cores scaling 2,
             i.e. a 100 % share: the tenant cannot lift its own limit any more, the plugin's
             limits file is the ceiling): the interception overhead alone — what the reference's vGPU column measured,
             whose 50 % SM limit did not bind (its vGPU numbers match native)
* vgpu-cu50  the contract exactly as emitted: 259 GiB oversubscribed quota (144 GiB of it
             HBM-resident), 128 of 256 CUs
* vdm        two pods of that plugin on one GPU running the same case concurrently
             (aggregate throughput; one GPU here, so 2 pods = the reference's 4 on 2 GPUs)

Statistics: --repeats R runs of native / vgpu / vgpu-cu50 in alternating (ABBA) order;
per case the overhead is the median over repeats of the paired ms/batch ratio, with a
95 % confidence interval (t-interval on the paired log-ratios).

    python benchmarks/aibench_suite.py [--cases all] [--repeats 5] [--steps 10 | --window SECONDS]
                                       [--json-out F] [--md-out F]
"""
import argparse
import json
import math
import os
import statistics
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

T95 = {1: 12.71, 2: 4.30, 3: 3.18, 4: 2.78, 5: 2.57, 6: 2.45, 7: 2.36, 8: 2.31, 9: 2.26, 10: 2.23}


def parse_cpulist(text):
    cpus = set()
    for part in text.strip().split(","):
        if "-" in part:
            lo, hi = part.split("-")
            cpus.update(range(int(lo), int(hi) + 1))
        elif part:
            cpus.add(int(part))
    return cpus


def gpu_local_cpus(bdf):
    """CPUs of the GPU's NUMA node that this process may run on (empty = do not pin).
    Launch-bound cases (small batches, thousands of kernels per step) run measurably
    slower from a remote NUMA node, which otherwise shows up as process-to-process
    jitter in both columns."""
    try:
        local = parse_cpulist(open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read())
    except (OSError, ValueError):
        return []
    return sorted(local & os.sched_getaffinity(0))


def worker(cases, steps, warmup, out, seconds=0.0, sync_dir=None, tag="0", peers=1, autotune=1):
    if os.environ.get("AIBENCH_CPUS"):
        os.sched_setaffinity(0, parse_cpulist(os.environ["AIBENCH_CPUS"]))
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = bool(autotune)  # MIOpen find mode (TF autotunes too)
    res = {}
    for name in cases:
        case = get_case(name)
        r = Runner(case, "cuda:0", dtype=torch.float32)
        for _ in range(warmup):
            r.step()
        torch.cuda.synchronize()
        if sync_dir:  # concurrent pods: every pod ready on this case, then go together
            open(os.path.join(sync_dir, f"{name}.{tag}"), "w").close()
            while len([f for f in os.listdir(sync_dir) if f.startswith(name + ".")]) < peers:
                time.sleep(0.002)
        n = 0
        t0 = time.perf_counter()
        while (n < steps) if not seconds else (time.perf_counter() - t0 < seconds):
            r.step()
            n += 1
            if seconds and n % 4 == 0:
                torch.cuda.synchronize()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        res[name] = {"ms_per_batch": dt * 1000 / n, "throughput": case.batch * n / dt, "batch": case.batch,
                     "steps": n}
        print(f"  [{tag}] {name}: {dt * 1000 / n:.3f} ms/batch", flush=True)
        del r
        torch.cuda.empty_cache()
    with open(out, "w") as f:
        json.dump(res, f)


AUTOTUNE = 1


def _cmd(cases, steps, warmup, out, extra=()):
    return [sys.executable, os.path.abspath(__file__), "--worker", "--cases", ",".join(cases), "--steps", str(steps),
            "--warmup", str(warmup), "--out", out, "--autotune", str(AUTOTUNE), *extra]


WINDOW = 0.0  # --window: each case timed over this many seconds instead of --steps


def run_mode(mode, node, uuid, cases, steps, warmup):
    from amdvgpu.shim.launcher import apply_contract
    fd, out = tempfile.mkstemp(suffix=".json")
    os.close(fd)
    if mode == "native":
        env = dict(os.environ, ROCR_VISIBLE_DEVICES=uuid)
    else:
        n = node[mode] if isinstance(node, dict) else node
        envs, mounts = n.pod(n.vgpu_ids(uuid)[:1])
        env = apply_contract(envs, mounts)
    print(f"[{mode}]", flush=True)
    try:
        extra = ["--seconds", str(WINDOW)] if WINDOW else []
        if subprocess.call(_cmd(cases, steps, warmup, out, extra), env=env):
            raise SystemExit(f"{mode} worker failed")
        return json.load(open(out))
    finally:
        os.unlink(out)


def l3_domain_of(cpu, allowed):
    """The CPUs sharing `cpu`'s L3 cache, within `allowed` (`allowed` if unknown)."""
    try:
        dom = parse_cpulist(open(f"/sys/devices/system/cpu/cpu{cpu}/cache/index3/shared_cpu_list").read())
    except OSError:
        return allowed
    return sorted(dom & set(allowed)) or allowed


def numa_cpus():
    """NUMA node -> the CPUs of it this process may use."""
    allowed = os.sched_getaffinity(0)
    out = {}
    base = "/sys/devices/system/node"
    for d in sorted(os.listdir(base)) if os.path.isdir(base) else []:
        if d.startswith("node") and d[4:].isdigit():
            try:
                cpus = parse_cpulist(open(os.path.join(base, d, "cpulist")).read()) & allowed
            except OSError:
                continue
            if cpus:
                out[int(d[4:])] = sorted(cpus)
    return out


def vdm_cpus(bdf, pods, placement):
    """Each VDM pod's CPUs. Two launch-bound processes whose threads run on one CPU socket do
    not run faster together than one alone on MI355X, while on two sockets they run at twice
    the rate (profiles/r5d). `product` (default) leaves the pods unpinned by the harness: the
    plugin's --numa-spread (default auto) gives the two vGPUs different CPU nodes and the shim
    keeps each pod there; `spread` pins pod i to NUMA node i mod nodes, GPU-local first, from
    here; `local` pins every pod to the GPU's node (round 4's setup)."""
    if placement in ("product", "none"):
        return [[] for _ in range(pods)]
    local = gpu_local_cpus(bdf)
    if placement == "local" or not local:
        return [local for _ in range(pods)]
    nodes = numa_cpus()
    order = [cs for cs in nodes.values() if set(cs) & set(local)] + \
            [cs for cs in nodes.values() if not set(cs) & set(local)]
    return [order[i % len(order)] for i in range(pods)]


VDM_PLACEMENT = "product"


def run_vdm(node, uuid, cases, warmup, seconds, pods=2, bdf=""):
    from amdvgpu.shim.launcher import apply_contract
    sync = tempfile.mkdtemp(prefix="vdm-")
    procs, outs = [], []
    cpus = vdm_cpus(bdf, pods, VDM_PLACEMENT)
    for i, vid in enumerate(node.vgpu_ids(uuid)[:pods]):
        envs, mounts = node.pod([vid])
        out = os.path.join(sync, f"res{i}.json")
        env = apply_contract(envs, mounts)
        env.pop("AIBENCH_CPUS", None)
        if cpus[i]:
            env["AIBENCH_CPUS"] = ",".join(map(str, cpus[i]))
        procs.append(subprocess.Popen(_cmd(cases, 0, warmup, out, ["--seconds", str(seconds), "--sync-dir", sync,
                                                                   "--tag", str(i), "--peers", str(pods)]),
                                      env=env))
        outs.append(out)
    print(f"[vdm x{pods}]", flush=True)
    for p in procs:
        if p.wait(timeout=3600):
            raise SystemExit("vdm pod failed")
    per = [json.load(open(o)) for o in outs]
    return {c: {"throughput": sum(p[c]["throughput"] for p in per), "per_pod": [p[c]["throughput"] for p in per]}
            for c in cases}


def ci_ratio(nat, vg):
    """Median paired ratio and 95 % CI (t-interval on log-ratios), as overhead percents."""
    lr = [math.log(v / n) for n, v in zip(nat, vg)]
    med = (math.exp(statistics.median(lr)) - 1) * 100
    if len(lr) < 2:
        return med, med, med
    m, sd = statistics.mean(lr), statistics.stdev(lr)
    h = T95.get(len(lr) - 1, 2.0) * sd / math.sqrt(len(lr))
    return med, (math.exp(m - h) - 1) * 100, (math.exp(m + h) - 1) * 100


def table(runs, vdm, cases):
    from amdvgpu.models.aibench import get_case
    lines = ["| test | case | batch | native ms/batch | vgpu ms/batch | vgpu overhead (median, 95 % CI) | "
             "reference vGPU overhead | vgpu-cu50 ms/batch | vdm (2 pods) throughput | V100 vGPU / vGPU+VDM |",
             "|---|---|---|---|---|---|---|---|---|---|"]
    summary = []
    for name in cases:
        c = get_case(name)
        nat = [r["native"][name]["ms_per_batch"] for r in runs]
        vg = [r["vgpu"][name]["ms_per_batch"] for r in runs]
        cu = [r["vgpu-cu50"][name]["ms_per_batch"] for r in runs if "vgpu-cu50" in r]
        med, lo, hi = ci_ratio(nat, vg)
        ref = (c.baseline_native / c.baseline_vgpu - 1) * 100
        summary.append({"case": name, "test": c.test_id, "native_ms": statistics.median(nat),
                        "vgpu_ms": statistics.median(vg), "overhead_pct": med, "ci95": [lo, hi],
                        "reference_overhead_pct": ref, "vgpu_cu50_ms": statistics.median(cu) if cu else None,
                        "vdm_throughput": vdm.get(name, {}).get("throughput") if vdm else None,
                        "repeats": len(nat)})
        vdm_s = f"{vdm[name]['throughput']:.1f} {c.unit}" if vdm and name in vdm else "-"
        cu_s = f"{statistics.median(cu):.2f}" if cu else "-"
        lines.append(f"| {c.test_id} | {name} | {c.batch} | {statistics.median(nat):.2f} | {statistics.median(vg):.2f} | "
                     f"{med:+.2f} % [{lo:+.2f}, {hi:+.2f}] | {ref:+.1f} % | {cu_s} | {vdm_s} | "
                     f"{c.baseline_vgpu} / {vdm_baseline(c)} |")
    ovs = sorted(s["overhead_pct"] for s in summary)
    if ovs:
        lines += ["", f"vGPU interception overhead over {len(runs)} ABBA repeats: median "
                      f"{statistics.median(ovs):+.2f} %, range {ovs[0]:+.2f} % .. {ovs[-1]:+.2f} % "
                      "(reference: median +2.5 %, range -3.8 % .. +17.7 %)"]
    return "\n".join(lines), summary


VDM_V100 = {"1.1": 207.9, "1.2": 79.84, "2.1": 211.3, "2.2": 45.14, "3.1": 179.77, "3.2": 14.87, "4.1": 11.1,
            "4.2": 7.69, "5.1": 23.02, "5.2": 6.95}


def vdm_baseline(c):
    return VDM_V100.get(c.test_id, "-")


def merge(paths, json_out, md_out):
    """One table over several suite runs (e.g. the two halves of the ten cases)."""
    from amdvgpu.models.aibench import CASES
    parts = [json.load(open(p)) for p in paths]
    n = min(len(p["runs"]) for p in parts)
    runs = [{} for _ in range(n)]
    vdm = {}
    for p in parts:
        for i in range(n):
            for mode, res in p["runs"][i].items():
                runs[i].setdefault(mode, {}).update(res)
        vdm.update(p.get("vdm") or {})
    have = set().union(*(r["native"].keys() for r in runs))
    cases = [c.name for c in sorted(CASES, key=lambda c: c.test_id) if c.name in have]
    md, summary = table(runs, vdm, cases)
    print(md)
    if json_out:
        json.dump({"merged": paths, "repeats": n, "summary": summary, "runs": runs, "vdm": vdm}, open(json_out, "w"),
                  indent=1)
    if md_out:
        open(md_out, "w").write(md + "\n")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--cases", default="all")
    ap.add_argument("--modes", default="native,vgpu,vgpu-cu50")
    ap.add_argument("--repeats", type=int, default=5)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--window", type=float, default=0.0,
                    help="time each case over this many seconds (every 4th step synchronised) instead of --steps")
    ap.add_argument("--vdm", type=int, default=1, help="also run the two-pod virtual-device-memory column")
    ap.add_argument("--vdm-seconds", type=float, default=3.0)
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--seconds", type=float, default=0.0)
    ap.add_argument("--sync-dir", default=None)
    ap.add_argument("--tag", default="0")
    ap.add_argument("--peers", type=int, default=1)
    ap.add_argument("--out", default=None)
    ap.add_argument("--json-out", default=None)
    ap.add_argument("--md-out", default=None)
    ap.add_argument("--merge", nargs="+", default=None,
                    help="render one table from the --json-out files of runs over disjoint case lists")
    ap.add_argument("--pin", type=int, default=1,
                    help="pin every worker to the GPU's NUMA-local CPUs (1), to one L3 domain of them (2), or not (0)")
    ap.add_argument("--vdm-placement", default="product", choices=["product", "spread", "local"],
                    help="CPUs of the two VDM pods: the plugin's --numa-spread places them (default), pinned one "
                         "per NUMA node from here, or both pinned GPU-local (round 4)")
    ap.add_argument("--autotune", type=int, default=1,
                    help="MIOpen find mode (cudnn.benchmark); 0 = deterministic heuristic solver choice")
    a = ap.parse_args()
    global AUTOTUNE, WINDOW, VDM_PLACEMENT
    AUTOTUNE = a.autotune
    VDM_PLACEMENT = a.vdm_placement
    WINDOW = a.window
    from amdvgpu.models.aibench import CASES
    cases = [c.name for c in CASES] if a.cases == "all" else a.cases.split(",")
    if a.worker:
        return worker(cases, a.steps, a.warmup, a.out, a.seconds, a.sync_dir, a.tag, a.peers, a.autotune)
    if a.merge:
        return merge(a.merge, a.json_out, a.md_out)
    from amdvgpu.plugin.devices import SysfsBackend
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    backend = SysfsBackend()
    dev = backend.devices()[0]
    uuid = dev.uuid
    cpus = gpu_local_cpus(dev.bdf) if a.pin else []
    if a.pin == 2 and cpus:
        # one L3 domain (CCD) of the GPU's node: launch-bound cases (thousands of kernels per
        # step) vary less from process to process when their threads stay on one CCD
        cpus = l3_domain_of(cpus[0], cpus)
    if cpus:
        os.environ["AIBENCH_CPUS"] = ",".join(map(str, cpus))
    print(f"GPU {dev.bdf}: workers pinned to {len(cpus)} NUMA-local CPUs" if cpus else "workers not pinned", flush=True)
    modes = a.modes.split(",")
    runs, vdm = [], {}
    # The reference's DaemonSet (split 2, memory scaling 1.8; no node bound on host memory, as
    # there), and the same at cores scaling 2 for the interception-only column.
    ref = dict(device_split_count=2, device_memory_scaling=1.8, host_memory_fraction=0.0)
    with NodeHarness(backend, **ref) as node, NodeHarness(backend, device_cores_scaling=2.0, **ref) as free:
        nodes = {"native": node, "vgpu": free, "vgpu-cu50": node}
        for rep in range(a.repeats):
            order = modes if rep % 2 == 0 else modes[::-1]  # ABBA: cancels drift between runs
            runs.append({m: run_mode(m, nodes, uuid, cases, a.steps, a.warmup) for m in order})
            if a.json_out:  # keep what is measured if a later step runs out of time
                json.dump({"steps": a.steps, "warmup": a.warmup, "repeats": rep + 1, "partial": True, "runs": runs},
                          open(a.json_out, "w"), indent=1)
        if a.vdm:
            vdm = run_vdm(node, uuid, cases, a.warmup, a.vdm_seconds, bdf=dev.bdf)
    md, summary = table(runs, vdm, cases)
    print(md)
    if a.json_out:
        json.dump({"steps": a.steps, "warmup": a.warmup, "repeats": a.repeats, "autotune": a.autotune,
                   "pinned_cpus": len(cpus), "vdm_placement": VDM_PLACEMENT, "summary": summary, "runs": runs,
                   "vdm": vdm}, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write(md + "\n")


if __name__ == "__main__":
    main()
