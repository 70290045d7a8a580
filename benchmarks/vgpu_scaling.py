#!/usr/bin/env python3
"""Concurrent-vGPU scaling curve on one MI355X: N pods (N = 1, 2, 4, 8) each running the
same stock workload (fp32, MIOpen / hipBLASLt) in its own vGPU, started together; reports
per-pod and aggregate throughput. This is the reference's "vGPU+VDM high load" column
(4 containers on 2 GPUs) generalised to the MI355X's tenant counts.

Every pod's contract comes from an Allocate of the plugin (NodeHarness, sysfs backend)
configured with --device-split-count=N and the policy's --cu-mode:

* default   --cu-mode auto (the shipped default): CU masks for 2 pods, the GPU-time
            limiter for 4 and 8
* spatial   --cu-mode spatial: disjoint XCD-balanced CU slices at every N
* temporal  --cu-mode temporal at every N
* shared    --cu-mode off: quota only, hardware time-sharing of all 256 CUs

    python benchmarks/vgpu_scaling.py [--case resnet50-inf] [--tenants 1,2,4,8] [--policy default,spatial,shared]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
HBM = 309220868096


def worker(case_name, steps, warmup, out, go_file, seconds):
    import faulthandler
    t_spawn = time.time()
    faulthandler.dump_traceback_later(200, exit=False)  # a pod stuck in warm-up shows where
    import torch
    from amdvgpu.models.aibench import Runner, get_case
    torch.backends.cudnn.benchmark = os.environ.get("VGPU_BENCH_AUTOTUNE", "1") != "0"  # MIOpen find mode
    case = get_case(case_name)
    t_import = time.time()
    r = Runner(case, "cuda:0", dtype=torch.float32)
    torch.cuda.synchronize()
    t_model = time.time()
    for i in range(warmup):
        r.step()
        if i == 0:
            torch.cuda.synchronize()
            t_first = time.time()
    torch.cuda.synchronize()
    import resource
    ru = resource.getrusage(resource.RUSAGE_SELF)  # every thread of the pod, start-up only
    startup = {"import_s": round(t_import - t_spawn, 2), "model_s": round(t_model - t_import, 2),
               "first_step_s": round(t_first - t_model, 2) if warmup else 0.0,
               "warmup_s": round(time.time() - (t_first if warmup else t_model), 2),
               "cpu_user_s": round(ru.ru_utime, 2), "cpu_sys_s": round(ru.ru_stime, 2),
               "max_rss_mb": round(ru.ru_maxrss / 1024, 1), "vol_ctx_switches": ru.ru_nvcsw}
    region = None
    if os.environ.get("VGPU_SHARED_CACHE") and os.path.exists(os.environ["VGPU_SHARED_CACHE"]):
        from amdvgpu.shim.region import Region
        region = Region(os.environ["VGPU_SHARED_CACHE"])
    faulthandler.cancel_dump_traceback_later()
    open(out + ".ready", "w").close()
    while not os.path.exists(go_file):
        time.sleep(0.005)
    g0 = region.device(0) if region else None
    # Waits block (interrupt-driven) instead of spinning: the box runs every pod in one CPU
    # quota (16 CPUs), where 16 spinning pods starve each other's launch threads; on a node
    # each pod spins on CPUs of its own. VGPU_BENCH_SYNC=spin restores torch's default wait.
    if os.environ.get("VGPU_BENCH_SYNC", "block") == "spin":
        sync = torch.cuda.synchronize
    else:
        def sync():
            ev = torch.cuda.Event(blocking=True)
            ev.record()
            ev.synchronize()
    ru0 = resource.getrusage(resource.RUSAGE_SELF)
    n = 0
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        r.step()
        n += 1
        if n % 4 == 0:
            sync()
    sync()
    t1 = time.perf_counter()
    ru1 = resource.getrusage(resource.RUSAGE_SELF)
    cpu_window = round(ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime, 2)
    threads = {}  # where the pod's CPU time went, by thread name (whole life: start-up included)
    tick = os.sysconf("SC_CLK_TCK")
    for t in os.listdir("/proc/self/task"):
        try:
            with open(f"/proc/self/task/{t}/stat") as f:
                st = f.read()
            name = st[st.index("(") + 1:st.rindex(")")]
            fields = st[st.rindex(")") + 2:].split()
            threads[name] = round(threads.get(name, 0.0) + (int(fields[11]) + int(fields[12])) / tick, 2)
        except (OSError, ValueError, IndexError):
            pass
    res = {"ms_per_batch": (t1 - t0) * 1000 / n, "t0": t0, "t1": t1, "batch": case.batch, "steps": n,
           "throughput": case.batch * n / (t1 - t0), "cu_mode": None, "crowd": None, "startup": startup,
           "cpu_s_in_window": cpu_window, "cpu_s_by_thread": threads}
    if region:
        g1 = region.device(0)  # the enforcement the pod ended under, and the GPU time it was charged
        res.update(cu_mode=g1["cu_mode"], crowd=g1["crowd"])
        if g1["wall_ns"] > g0["wall_ns"]:
            charged_ms = (g1["charged_ns"] - g0["charged_ns"]) / 1e6
            res["gpu_ms_charged"] = round(charged_ms, 2)
            res["granted_pct"] = round(100.0 * (g1["charged_ns"] - g0["charged_ns"]) / (g1["wall_ns"] - g0["wall_ns"]), 2)
            if charged_ms > 0:  # throughput per charged GPU-millisecond (profiles/r2ak)
                res["images_per_gpu_ms"] = round(case.batch * n / charged_ms, 4)
        region.close()
    json.dump(res, open(out, "w"))


MODES = {"default": "auto", "spatial": "spatial", "temporal": "temporal", "shared": "off"}


def kfd_queue_count():
    """User-mode queues of every process on the node's GPUs (KFD sysfs), or None."""
    root = "/sys/class/kfd/kfd/proc"
    try:
        return sum(len(os.listdir(os.path.join(root, p, "queues"))) for p in os.listdir(root)
                   if os.path.isdir(os.path.join(root, p, "queues")))
    except OSError:
        return None


def stuck_report(outs, regions, procs):
    """Which pods never got ready, and what their regions say (limiter state, gates)."""
    from amdvgpu.shim.region import Region
    for o, reg, p in zip(outs, regions, procs):
        if os.path.exists(o + ".ready"):
            continue
        info = {"pod": os.path.basename(o), "pid": p.pid, "exit": p.poll()}
        try:
            with Region(reg) as r:
                snap = r.snapshot()
            d = snap["devices"][0] if snap["devices"] else {}
            info.update(suspended=snap["suspended"], recent_kernel=snap["recent_kernel"], samples=snap["samples"],
                        credit_ms=d.get("credit_ns", 0) / 1e6, cu_mode=d.get("cu_mode"), crowd=d.get("crowd"),
                        util_pct=d.get("util_pct"), procs=[{k: q[k] for k in ("pid", "hostpid", "launches",
                                                                            "throttle_ns", "status")}
                                                           for q in snap["procs"]])
        except OSError as e:
            info["region_error"] = str(e)
        try:
            with open(f"/proc/{p.pid}/wchan") as f:
                info["wchan"] = f.read().strip()
            info["threads"] = {}
            for t in os.listdir(f"/proc/{p.pid}/task"):
                with open(f"/proc/{p.pid}/task/{t}/wchan") as f:
                    w = f.read().strip()
                with open(f"/proc/{p.pid}/task/{t}/comm") as f:
                    c = f.read().strip()
                info["threads"][f"{t}:{c}"] = w
        except OSError:
            pass
        print("STUCK " + json.dumps(info), flush=True)


def miopen_dirs(mode, tmp, i):
    """MIOpen's find-db and kernel cache for pod ``i``. ``home``: the process's default
    (~/.config/miopen, ~/.cache/miopen: one set for every pod on this box - pods of a real node
    each have their own filesystem); ``per-pod``: the pod's own copy of the default set (an
    image that ships a tuned find-db); ``empty``: the pod's own empty set (a pod's first run)."""
    if mode == "home":
        return {}
    import shutil
    base = os.path.join(tmp, f"miopen{i}")
    db, cache = os.path.join(base, "db"), os.path.join(base, "cache")
    home = os.path.expanduser("~")
    src_db, src_cache = os.path.join(home, ".config", "miopen"), os.path.join(home, ".cache", "miopen")
    if mode == "per-pod" and os.path.isdir(src_db):
        shutil.copytree(src_db, db)
    if mode == "per-pod" and os.path.isdir(src_cache):
        shutil.copytree(src_cache, cache)
    os.makedirs(db, exist_ok=True)
    os.makedirs(cache, exist_ok=True)
    return {"MIOPEN_USER_DB_PATH": db, "MIOPEN_CUSTOM_CACHE_DIR": cache}


def run_point(backend, uuid, case, n, policy, warmup, seconds, hw_queues=0, pod_env=None, split=0, ledger=None,
              miopen="home", conc=None):
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    from amdvgpu.shim.launcher import apply_contract
    tmp = tempfile.mkdtemp(prefix="scal-")
    go = os.path.join(tmp, "go")
    procs, outs, regions = [], [], []
    kw = {} if ledger is None else {"ledger": bool(ledger)}
    if conc is not None:
        kw["gpu_concurrency"] = conc
    with NodeHarness(backend, device_split_count=split or n, cu_mode=MODES[policy], **kw) as node:
        for i, vid in enumerate(node.vgpu_ids(uuid)[:n]):
            envs, mounts = node.pod([vid])
            out = os.path.join(tmp, f"t{i}.json")
            cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--case", case, "--warmup", str(warmup),
                   "--seconds", str(seconds), "--out", out, "--go", go]
            env = apply_contract(envs, mounts)
            regions.append(env.get("VGPU_SHARED_CACHE"))
            if hw_queues:
                env["GPU_MAX_HW_QUEUES"] = str(hw_queues)
            env.update(pod_env or {})
            env.update(miopen_dirs(miopen, tmp, i))
            procs.append(subprocess.Popen(cmd, env=env))
            outs.append(out)
        try:
            t_start = beat = time.time()
            deadline = t_start + 300
            while not all(os.path.exists(o + ".ready") for o in outs):
                if any(p.poll() not in (None, 0) for p in procs) or time.time() > deadline:
                    stuck_report(outs, regions, procs)
                    raise SystemExit("a tenant failed before the start barrier")
                if time.time() - beat > 30:
                    beat = time.time()
                    print(f"  waiting: {sum(os.path.exists(o + '.ready') for o in outs)}/{n} pods warmed up",
                          flush=True)
                time.sleep(0.05)
            warm_s = time.time() - t_start
            queues = kfd_queue_count()
            open(go, "w").close()
            for p in procs:
                if p.wait(timeout=900) != 0:
                    raise SystemExit("a tenant failed")
            res = [json.load(open(o)) for o in outs]
        finally:
            for p in procs:
                if p.poll() is None:
                    p.kill()
    span = max(r["t1"] for r in res) - min(r["t0"] for r in res)
    agg = sum(r["batch"] * r["steps"] for r in res) / span
    import shutil
    shutil.rmtree(tmp, ignore_errors=True)
    return {"tenants": n, "policy": policy, "split": split or n, "hw_queues": hw_queues or None, "kfd_queues": queues,
            "miopen_db": miopen, "startup": [r.get("startup") for r in res],
            "warmup_s": round(warm_s, 1), "pod_env": pod_env or None, "modes": sorted({str(r.get("cu_mode")) for r in res}),
            "aggregate_throughput": agg,
            "per_tenant": [r["throughput"] for r in res], "per_tenant_ms": [r["ms_per_batch"] for r in res],
            "per_tenant_granted_pct": [r.get("granted_pct") for r in res],
            "per_tenant_images_per_gpu_ms": [r.get("images_per_gpu_ms") for r in res],
            "per_tenant_cpu_s": [r.get("cpu_s_in_window") for r in res],
            "cpu_s_by_thread": [r.get("cpu_s_by_thread") for r in res]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--case", default="resnet50-inf")
    ap.add_argument("--tenants", default="1,2,4,8")
    ap.add_argument("--policy", default="default,spatial,shared")
    ap.add_argument("--seconds", type=float, default=6.0)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--hw-queues", default="0", help="GPU_MAX_HW_QUEUES per pod (comma list; 0 = HIP default)")
    ap.add_argument("--pod-env", action="append", default=[],
                    help="KEY=V1,V2,...: extra env in every pod, one sweep per value (repeatable)")
    ap.add_argument("--repeats", type=int, default=1)
    ap.add_argument("--split", type=int, default=0, help="vGPUs per GPU (default: one per pod)")
    ap.add_argument("--node-ledger", type=int, choices=[0, 1], default=None,
                    help="1/0: the plugin runs the node GPU-time ledger (vgpu-ledger) or not (default: the "
                    "plugin's default, on)")
    ap.add_argument("--miopen-db", default="home", choices=["home", "per-pod", "empty"],
                    help="MIOpen find-db / kernel cache of the pods (see miopen_dirs)")
    ap.add_argument("--gpu-concurrency", type=lambda v: -1 if v == "auto" else int(v), default=None,
                    help="the plugin's --gpu-concurrency (default: the plugin's own default)")
    ap.add_argument("--worker", action="store_true")
    ap.add_argument("--out")
    ap.add_argument("--go")
    ap.add_argument("--json-out")
    ap.add_argument("--md-out")
    a = ap.parse_args()
    if a.worker:
        return worker(a.case, 0, a.warmup, a.out, a.go, a.seconds)
    from amdvgpu.plugin.devices import SysfsBackend
    backend = SysfsBackend()
    uuid = backend.devices()[0].uuid
    rows = []
    envs = [{}]
    for spec in a.pod_env:
        k, _, vals = spec.partition("=")
        envs = [dict(e, **{k: v}) for e in envs for v in vals.split(",")]
    for rep in range(a.repeats):
        for k, pe in enumerate(envs):
            for hq in [int(x) for x in a.hw_queues.split(",")]:
                for pol in a.policy.split(","):
                    for n in [int(x) for x in a.tenants.split(",")]:
                        # The lone pod is the whole-GPU reference point: run once per
                        # repeat, without the pod env under study.
                        if n == 1 and k > 0:
                            continue
                        r = run_point(backend, uuid, a.case, n, pol, a.warmup, a.seconds, hq,
                                      pe if n > 1 else None, a.split, ledger=a.node_ledger,
                                      miopen=a.miopen_db if n > 1 else "home", conc=a.gpu_concurrency)
                        rows.append(r)
                        print(json.dumps(r), flush=True)
    base = {r["policy"]: r["aggregate_throughput"] for r in rows if r["tenants"] == 1}
    md = [f"# concurrent vGPU pods on one MI355X — {a.case} (stock fp32; contracts from Allocate)", "",
          "| policy (--cu-mode) | split | enforcement | pod env | HW queues/pod | KFD queues | pods | aggregate | "
          "vs 1 pod | per pod (min..max) | slowest pod vs 1/N of one pod (fixed --split: vs the lone pod) |",
          "|---|---|---|---|---|---|---|---|---|---|---|"]
    for r in rows:
        pt = r["per_tenant"]
        b = base.get(r["policy"])  # no 1-pod run of this policy in the sweep: no ratios
        pe = " ".join(f"{k}={v}" for k, v in (r["pod_env"] or {}).items()) or "-"
        vs_one = f"{r['aggregate_throughput'] / b:.2f}x" if b else "n/a"
        slowest = f"{min(pt) / (b / (r['tenants'] if r['split'] == r['tenants'] else 1)):.2f}" if b else "n/a"
        md.append(f"| {r['policy']} ({MODES[r['policy']]}) | {r['split']} | {'/'.join(r['modes'])} | {pe} | "
                  f"{r['hw_queues'] or 'default'} | {r['kfd_queues']} | "
                  f"{r['tenants']} | {r['aggregate_throughput']:.1f} | "
                  f"{vs_one} | {min(pt):.1f} .. {max(pt):.1f} | {slowest} |")
    print("\n".join(md))
    if a.json_out:
        json.dump(rows, open(a.json_out, "w"), indent=1)
    if a.md_out:
        open(a.md_out, "w").write("\n".join(md) + "\n")


if __name__ == "__main__":
    main()
