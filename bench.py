#!/usr/bin/env python3
"""Headline benchmark: stock PyTorch-ROCm ResNet-V2-50 inference (ai-benchmark test 1.1,
batch 50, 346², fp32) inside a vGPU of one MI355X, as the device plugin allocates it.

BASELINE.json config 2 (split 4, 72 GiB quota per pod) with the reference's metric: the
ms/batch cost of the vGPU versus native, and how many vGPUs one GPU sustains.

Every vGPU contract comes from a real ``Allocate`` call: the plugin (``main.Supervisor``
on the sysfs device backend) registers with a stub kubelet, the rank's GPU is allocated,
and the returned envs + mounts are applied to the worker process exactly as a container
runtime would (``shim/launcher.py``), so the workload runs under the interception shim
(``libvgpu_hip.so``) with the limits a pod would get. The workload is stock PyTorch
(MIOpen / hipBLASLt kernels, no custom fused ops) in fp32, the reference's precision.

Modes, one fresh worker process each (the rank process itself never touches the GPU):

* native   no shim; the GPU made visible as the official plugin would.
* vgpu     the split-4 pod: 72 GiB quota, 25 % compute share. Auto mode enforces it with
           the pod's 64-CU mask while the GPU is not crowded (here the pod is alone),
           and with the GPU-time limiter once two or more other processes keep the GPU
           busy (the sweep's 4 and 8 pods). The line reports the enforcement used
           (``effective_cu_mode``, ``crowd``).   → ``value``
* quota    the same pod without a compute limit (the plugin at cores scaling = split): the
           shim's own overhead on stock PyTorch, the number the reference's vGPU column
           measured (its 50 % SM limit did not bind on TF).
* parity   the reference's benchmark configuration: split 2, memory scaling 1.8
           (server.go:492,505-507): 50 % compute (CU mask), 259 GiB oversubscribed quota.
* sweep    N = 1, 2, 4, 8, 12 pods of a split-N plugin run concurrently on one GPU
           (default deployment config). ``max_vgpus_per_gpu`` is the largest N whose
           aggregate stays >= 0.9x one whole-GPU pod and whose slowest pod gets >= 0.9x
           its 1/N entitlement. Only on single-GPU runs unless --sweep on. The whole run
           takes about 8 minutes, 12 pods about 3 of them (mostly the pods' start-up).
           ``--time-budget`` (default 540 s) bounds the run: a point whose estimated
           duration would overrun it is skipped and listed as such in ``sweep``.
* node     BASELINE config 5: all --split vGPUs of every GPU of the job busy at once
           (32 vGPUs on an 8-GPU node), released together across the ranks. Reported as
           ``node``: the aggregate over every vGPU, vs native x GPUs, and the slowest pod
           vs its 1/split entitlement. Runs on multi-GPU jobs; a single-GPU run takes it
           from the sweep's --split point.

Timed region (native / vgpu / quota / parity): W untimed warmup steps, then exactly K
steps bracketed by barrier + synchronize on both sides; MAX step time over ranks (one
rank per GPU under torch.distributed.run; the pods are independent tenants, so the
cross-rank group is gloo). ``value`` is the whole-job vGPU throughput (sum over GPUs).
With N > 1 an RCCL all-reduce between the ranks' pods is probed afterwards, natively and
inside the pods, and its bus bandwidth compared (``rccl_allreduce_between_pods``).

Ranks: under torch.distributed.run each rank takes its GPU from LOCAL_RANK. Called as
``python bench.py --gpus N`` (N > 1) with no launcher, the process starts the N ranks
itself (torch.distributed.run on 127.0.0.1, before anything touches a GPU) and exits with
their code, so the line always covers the N GPUs it names; N beyond the GPUs the job can
see (render nodes it may open, ROCR/HIP_VISIBLE_DEVICES) is refused with a non-zero exit.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--case resnet50-inf] [--sweep auto|on|off]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

T_START = time.time()
REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

METRIC = ("ai-benchmark ResNet-50 ms/batch overhead vs native plugin; max vGPUs per MI355X "
          "(value: ResNet-V2-50 b=50 346² fp32 inference throughput inside a split-4 vGPU, images/s)")
SWEEP_MIN_AGGREGATE = 0.9
SWEEP_MIN_TENANT = 0.9


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--case", default="resnet50-inf")
    ap.add_argument("--modes", default="native,vgpu,quota,parity")
    ap.add_argument("--split", type=int, default=4, help="vGPUs per GPU of the headline pod (BASELINE config 2)")
    ap.add_argument("--cu-mode", default="auto", choices=["auto", "spatial", "temporal", "both", "off"])
    ap.add_argument("--dtype", default="fp32", choices=["fp32", "bf16"])
    ap.add_argument("--sweep", default="auto", choices=["auto", "on", "off"])
    ap.add_argument("--sweep-tenants", default="1,2,4,8,12,16")
    ap.add_argument("--sweep-seconds", type=float, default=6.0)
    ap.add_argument("--sweep-autotune", type=int, default=0,
                    help="1: every sweep pod runs MIOpen's find (benchmark mode) at start-up; 0 (default): the "
                         "sweep's pods, the lone one included, use MIOpen's immediate mode - the same ResNet-50 "
                         "throughput on MI355X (3747 vs 3741 img/s alone) without 16 concurrent searches "
                         "(a 16-pod point starts in 15 s instead of ~150 s, profiles/r4l)")
    ap.add_argument("--sweep-find-db", default="per-pod", choices=["per-pod", "home", "empty"],
                    help="MIOpen find-db and kernel cache of the sweep's pods: per-pod = each pod its own copy "
                         "of what the lone pod left (a tenant image that ships a tuned find-db; pods of a node "
                         "never share one file system); home = this process's own (~/.config/miopen: one sqlite "
                         "set shared by every pod on this box); empty = each pod its own empty set (a pod's "
                         "first run: every pod runs its own find)")
    ap.add_argument("--sweep-pod-env", action="append", default=[],
                    help="KEY=VALUE added to the env of every sweep pod (studies; repeatable)")
    ap.add_argument("--node", default="auto", choices=["auto", "on", "off"],
                    help="node point: all --split vGPUs of every GPU of the job busy at once (BASELINE config 5: "
                         "32 vGPUs on 8 GPUs); auto = on for multi-GPU runs (single-GPU runs take it from the sweep)")
    ap.add_argument("--time-budget", type=float, default=540.0,
                    help="wall seconds for the whole run: sweep points that would not finish in time are "
                         "skipped (and reported as such), so the line is always printed")
    ap.add_argument("--ledger", action=argparse.BooleanOptionalAction, default=None,
                    help="the plugin runs the node GPU-time ledger (exact charges and shares; default: the "
                         "plugin's own default)")
    ap.add_argument("--json-out", default=None, help="also write the result line to this file")
    ap.add_argument("--rccl-probe", type=int, default=1, help="N>1: RCCL all-reduce between the pods afterwards")
    # worker-only
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mode", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--result-file", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--port", type=int, default=0, help=argparse.SUPPRESS)
    ap.add_argument("--dist", type=int, default=1, help=argparse.SUPPRESS)
    ap.add_argument("--seconds", type=float, default=0.0, help=argparse.SUPPRESS)
    ap.add_argument("--go", default=None, help=argparse.SUPPRESS)
    # CPU rehearsal of the multi-rank orchestration (gloo, fake devices, tiny input); not a measurement
    ap.add_argument("--cpu-rehearsal", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- worker


def worker(args):
    t_spawn = time.time()
    import torch
    import torch.distributed as dist

    from amdvgpu.models.aibench import Runner, get_case
    phases = {"import_s": time.time() - t_spawn}

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1)) if args.dist else 1
    cpu = args.cpu_rehearsal
    # The pod sees exactly its own GPU (ROCR_VISIBLE_DEVICES from the contract): cuda:0.
    device = torch.device("cpu") if cpu else torch.device("cuda", 0)
    if not cpu:
        torch.cuda.set_device(device)
        torch.zeros(1, device=device)  # HIP / ROCr (and the shim) initialised here
    phases["gpu_init_s"] = time.time() - t_spawn - sum(phases.values())
    if world > 1:
        # The pods are independent tenants (no gradient exchange): the cross-rank group only
        # brackets the timed window and takes the max, so it runs on gloo over TCP and the
        # measurement cannot depend on GPU peer access between pods. RCCL through the shim
        # is exercised separately (mode "rccl").
        init = f"tcp://{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{args.port}"
        dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    if args.mode == "rccl":
        return rccl_probe(args, device, rank, world)
    if cpu and args.mode == "node" and os.environ.get("VGPU_BENCH_FAIL_NODE_RANK") == str(rank):
        raise SystemExit("rehearsal: this rank's node pods fail")  # tests/test_bench_contract.py
    sync = (lambda: None) if cpu else (lambda: torch.cuda.synchronize(device))
    free0, total = torch.cuda.mem_get_info(device) if not cpu else (0, 0)
    quota = int(os.environ.get("VGPU_DEVICE_MEMORY_LIMIT_0", "0").rstrip("m") or 0) << 20
    if quota and not cpu and total != quota:
        raise SystemExit(f"vGPU shim not in effect: mem_get_info total {total} != quota {quota}")

    # MIOpen find mode (the reference's TF autotunes too); --sweep-autotune 0 gives the sweep's
    # pods MIOpen's immediate mode (no per-process search) - the lone pod included.
    torch.backends.cudnn.benchmark = not (args.go and not args.sweep_autotune)
    case = get_case(args.case)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    if cpu:
        runner = Runner(case, device, dtype=torch.float32, batch=2, channels_last=False)
        runner.x = runner.x[..., :64, :64].contiguous() if runner.x.dim() == 4 else runner.x[:, :16].contiguous()
    else:
        runner = Runner(case, device, dtype=dtype)
    sync()
    phases["model_s"] = time.time() - t_spawn - sum(phases.values())
    for i in range(args.warmup):
        runner.step()
        if i == 0:
            sync()
            phases["first_step_s"] = time.time() - t_spawn - sum(phases.values())
    sync()
    phases["warmup_s"] = time.time() - t_spawn - sum(phases.values())
    if args.go:  # where a pod's start-up goes (many-pod sweep points are dominated by it)
        print("[bench-worker] start-up " + json.dumps({k: round(v, 2) for k, v in phases.items()}), file=sys.stderr,
              flush=True)

    def barrier():
        sync()
        if world > 1:
            dist.barrier()

    if args.go:  # concurrent tenants: start together, run for a fixed wall time
        open(args.result_file + ".ready", "w").close()
        while not os.path.exists(args.go):
            time.sleep(0.002)
        # How a pod waits for its GPU work. The default, spin, is a stock tenant's: torch's
        # synchronize every 4 steps. HIP spins a core through it (profiles/r4za); on a crowded
        # GPU the shim turns that wait into polling with short sleeps (sync_hooks.cpp,
        # profiles/r5c), so 16 waiting pods do not starve the ones that have work to launch.
        # VGPU_BENCH_SYNC=poll: the harness polls itself (3 steps in flight, 0.5 ms sleeps
        # between event queries; round 4's default); block: a blocking event wait every 4
        # steps.
        sync_mode = "cpu" if cpu else os.environ.get("VGPU_BENCH_SYNC", "spin")
        if sync_mode == "block":
            def wait():
                ev = torch.cuda.Event(blocking=True)
                ev.record()
                ev.synchronize()
        elif sync_mode == "poll":
            def wait():
                for e in marks:
                    while not e.query():
                        time.sleep(0.0005)
        else:
            wait = sync
        # When each step finished, on this process's perf_counter clock (shared by the pods of
        # a host): a timing event after every step, read back once at the end, so the parent
        # can rate every pod over the window in which all of them run (common_window()).
        import resource
        # The limiter's account of the window, read from the pod's region like vgpuctl: the
        # GPU time charged to the pod and the enforcement it ran under (why a pod falls behind)
        region = None
        if not cpu and os.environ.get("VGPU_SHARED_CACHE") and os.path.exists(os.environ["VGPU_SHARED_CACHE"]):
            from amdvgpu.shim.region import Region
            region = Region(os.environ["VGPU_SHARED_CACHE"])
        g0 = region.device(0) if region else None
        th0 = sum(p["throttle_ns"] for p in region.procs()) if region else 0
        marks = []
        n = 0
        ru0 = resource.getrusage(resource.RUSAGE_SELF)
        t0 = time.perf_counter()
        if not cpu:
            ev0 = torch.cuda.Event(enable_timing=True)
            ev0.record()
        while time.perf_counter() - t0 < args.seconds:
            runner.step()
            n += 1
            if cpu:
                marks.append(time.perf_counter())
            else:
                marks.append(torch.cuda.Event(enable_timing=True))
                marks[-1].record()
            if sync_mode == "poll":
                if n > 3:
                    while not marks[n - 4].query():
                        time.sleep(0.0005)
            elif n % 4 == 0:
                wait()
        wait()
        dt = time.perf_counter() - t0
        ru1 = resource.getrusage(resource.RUSAGE_SELF)
        done = marks if cpu else [t0 + ev0.elapsed_time(e) / 1000.0 for e in marks]
        res = {"mode": args.mode, "ms_per_step": dt * 1000.0 / n, "items_per_step": runner.items_per_step,
               "steps": n, "t0": t0, "t1": t0 + dt, "step_done": done, "wait": sync_mode,
               # CPU seconds of every thread of the pod in its window (the box runs all pods in
               # one 16-CPU quota: a point whose pods need more is CPU-bound, not GPU-bound)
               "cpu_s": round(ru1.ru_utime + ru1.ru_stime - ru0.ru_utime - ru0.ru_stime, 3),
               "startup": {k: round(v, 2) for k, v in phases.items()}}
        g1 = region.device(0) if region else None
        if g0 and g1 and g1["wall_ns"] > g0["wall_ns"]:
            res["granted_pct"] = round(100.0 * (g1["charged_ns"] - g0["charged_ns"]) / (g1["wall_ns"] - g0["wall_ns"]), 2)
            res["cu_mode_end"] = g1["cu_mode"]
            res["crowd_end"] = g1["crowd"]
            # time this pod's launches waited at the limiter's gate, % of the window
            res["throttled_pct"] = round(100.0 * (sum(p["throttle_ns"] for p in region.procs()) - th0) /
                                         (g1["wall_ns"] - g0["wall_ns"]), 2)
            # the processes the pod's limiter charges for (container pid, host pid)
            res["region_procs"] = [[p["pid"], p["hostpid"]] for p in region.procs()] + [["self", os.getpid()]]
        if region:
            region.close()
    else:
        # The limiter's own account of the timed window (GPU time charged / wall time), read
        # from the pod's shared region like vgpuctl would: what the vGPU granted this pod.
        region = None
        if not cpu and os.environ.get("VGPU_SHARED_CACHE") and os.path.exists(os.environ["VGPU_SHARED_CACHE"]):
            from amdvgpu.shim.region import Region
            region = Region(os.environ["VGPU_SHARED_CACHE"])
        barrier()
        g0 = region.device(0) if region else None
        t0 = time.perf_counter()
        for _ in range(args.steps):
            runner.step()
        sync()
        barrier()
        dt = time.perf_counter() - t0
        g1 = region.device(0) if region else None
        ms = torch.tensor([dt * 1000.0 / args.steps], dtype=torch.float64)
        if world > 1:
            dist.all_reduce(ms, op=dist.ReduceOp.MAX)
        res = {"mode": args.mode, "ms_per_step": ms.item(), "items_per_step": runner.items_per_step,
               "steps": args.steps, "mem_total": total,
               "peak_allocated": torch.cuda.max_memory_allocated(device) if not cpu else 0}
        if g1:
            # The enforcement the pod actually ran under (auto mode: CU mask when the GPU is
            # not crowded, GPU-time limiter when it is) and the crowd it saw.
            res["effective_cu_mode"] = g1["cu_mode"]
            res["crowd"] = g1["crowd"]
        if g0 and g1 and g1["wall_ns"] > g0["wall_ns"]:
            res["limiter_granted_pct"] = round(100.0 * (g1["charged_ns"] - g0["charged_ns"]) /
                                               (g1["wall_ns"] - g0["wall_ns"]), 2)
            res["gpu_ms_charged_per_step"] = round((g1["charged_ns"] - g0["charged_ns"]) / 1e6 / args.steps, 3)
        if region:
            region.close()
    if args.result_file and (rank == 0 or world == 1):
        with open(args.result_file, "w") as f:
            json.dump(res, f)
    if world > 1:
        barrier()
        dist.destroy_process_group()
    return 0


def rccl_probe(args, device, rank, world):
    """RCCL all-reduce between the ranks' vGPU pods, through the shim (IPC / peer access
    must pass untouched and imports must not be charged twice). Reports bus bandwidth;
    runs after the measurement in its own process, bounded by the parent's timeout."""
    import torch
    import torch.distributed as dist
    cpu = args.cpu_rehearsal
    pg = dist.new_group(backend="gloo" if cpu else "nccl")
    sync = (lambda: None) if cpu else (lambda: torch.cuda.synchronize(device))
    total = torch.cuda.mem_get_info(device)[1] if not cpu else 0
    n = (1 << 16) if cpu else (64 << 20)  # 64 Mi floats = 256 MiB per rank
    x = torch.full((n,), float(rank + 1), device=device)
    dist.all_reduce(x, group=pg)
    sync()
    ok = bool(torch.allclose(x[:1024], torch.full((1024,), world * (world + 1) / 2.0, device=device)))
    iters = 10
    t0 = time.perf_counter()
    for _ in range(iters):
        dist.all_reduce(x, group=pg)
    sync()
    dt = (time.perf_counter() - t0) / iters
    busbw = 2 * (world - 1) / world * n * 4 / dt / 1e9
    res = {"ok": ok, "backend": "gloo (cpu rehearsal)" if cpu else "nccl (RCCL)", "bytes": n * 4,
           "ms": round(dt * 1000, 3), "busbw_GBps": round(busbw, 3), "mem_get_info_total": total}
    if args.result_file and rank == 0:
        with open(args.result_file, "w") as f:
            json.dump(res, f)
    dist.destroy_process_group()
    return 0


# ----------------------------------------------------------------------------- parent


def worker_cmd(args, mode, result, port, dist=1, seconds=0.0, go=None):
    cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--mode", mode, "--result-file", result,
           "--port", str(port), "--dist", str(dist), "--case", args.case, "--steps", str(args.steps),
           "--warmup", str(args.warmup), "--dtype", args.dtype]
    if args.cpu_rehearsal:
        cmd.append("--cpu-rehearsal")
    if go:
        cmd += ["--seconds", str(seconds), "--go", go, "--sweep-autotune", str(args.sweep_autotune)]
    return cmd


def plugin_default_ledger():
    from amdvgpu.plugin.config import PluginConfig
    return PluginConfig().ledger


def ledger_kw(args):
    """NodeHarness keyword for --ledger / --no-ledger (none: the plugin's default)."""
    return {} if args.ledger is None else {"ledger": args.ledger}


# The job's own device selection (e.g. HIP_VISIBLE_DEVICES=0..7 on an 8-GPU node) indexes
# the node's GPUs; inside a pod (ROCR_VISIBLE_DEVICES = its GPU) those indices mean nothing.
HOST_SELECTORS = ("HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES", "GPU_DEVICE_ORDINAL")


def pod_env(node, ids, extra=None):
    """(process env, contract envs) for a container holding vGPUs ``ids``."""
    from amdvgpu.shim.launcher import apply_contract
    envs, mounts = node.pod(ids)
    env = apply_contract(envs, mounts)
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    for k in HOST_SELECTORS:  # a container starts without the host job's device selection
        env.pop(k, None)
    if extra:
        env.update(extra)
    return env, envs


def native_env(uuid, cpu):
    env = dict(os.environ)
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    for k in HOST_SELECTORS:
        env.pop(k, None)
    if not cpu:
        env["ROCR_VISIBLE_DEVICES"] = uuid  # the official plugin exposes the GPU the same way
    return env


def run_one(args, mode, env, port):
    """One timed worker (all ranks take part in its process group). Rank 0 returns the
    result dict, other ranks None."""
    fd, result = tempfile.mkstemp(prefix=f"bench-{mode}-", suffix=".json")
    os.close(fd)
    try:
        t0 = time.time()
        rc = subprocess.call(worker_cmd(args, mode, result, port), env=env)
        if rc != 0:
            raise SystemExit(f"bench worker ({mode}) failed with exit code {rc}")
        print(f"[bench] {mode}: worker done in {time.time() - t0:.0f} s", file=sys.stderr, flush=True)
        if int(os.environ.get("RANK", 0)) != 0:
            return None
        with open(result) as f:
            return json.load(f)
    finally:
        os.unlink(result)


def probe_rccl(args, env, port, timeout=120):
    """RCCL all-reduce across the ranks' vGPU pods (never fails the bench: a failure or
    timeout is reported as such)."""
    fd, result = tempfile.mkstemp(prefix="bench-rccl-", suffix=".json")
    os.close(fd)
    p = subprocess.Popen(worker_cmd(args, "rccl", result, port), env=env)
    try:
        rc = p.wait(timeout=timeout)
    except subprocess.TimeoutExpired:
        p.kill()
        p.wait()
        rc = "timeout"
    try:
        if rc != 0:
            return {"ok": False, "error": f"exit {rc}"}
        if int(os.environ.get("RANK", 0)) != 0:
            return None
        with open(result) as f:
            return json.load(f)
    except (OSError, ValueError) as e:
        return {"ok": False, "error": repr(e)[:200]}
    finally:
        os.unlink(result)


def now():
    return time.time()


class OutOfTime(Exception):
    pass


def run_concurrent(args, envs, label, deadline=None, before_go=None):
    """Starts one tenant per env, releases them together, returns their results. Raises
    OutOfTime when the tenants are not all warmed up by ``deadline`` (epoch seconds).
    ``before_go`` runs once every tenant is warmed up, right before the release (the node
    point's cross-rank barrier, so the pods of every GPU run in the same window)."""
    tmp = tempfile.mkdtemp(prefix=f"bench-{label}-")
    go = os.path.join(tmp, "go")
    procs, outs = [], []
    for i, env in enumerate(envs):
        out = os.path.join(tmp, f"t{i}.json")
        procs.append(subprocess.Popen(worker_cmd(args, label, out, 0, dist=0, seconds=args.sweep_seconds, go=go),
                                      env=env))
        outs.append(out)
    try:
        t_start = beat = time.time()
        deadline = deadline or t_start + 900
        while not all(os.path.exists(o + ".ready") for o in outs):
            if any(p.poll() not in (None, 0) for p in procs):
                raise SystemExit(f"a {label} tenant failed before the start barrier")
            if time.time() > deadline:
                raise OutOfTime(f"{sum(os.path.exists(o + '.ready') for o in outs)}/{len(outs)} tenants warmed up "
                                f"after {time.time() - t_start:.0f} s")
            if time.time() - beat > 30:
                beat = time.time()
                print(f"[bench] {label}: {sum(os.path.exists(o + '.ready') for o in outs)}/{len(outs)} tenants "
                      f"warmed up after {beat - t_start:.0f} s", file=sys.stderr, flush=True)
            time.sleep(0.05)
        print(f"[bench] {label}: all {len(outs)} tenants warmed up after {time.time() - t_start:.0f} s",
              file=sys.stderr, flush=True)
        if before_go:
            before_go()
        open(go, "w").close()
        for p in procs:
            if p.wait(timeout=900) != 0:
                raise SystemExit(f"a {label} tenant failed")
        return [json.load(open(o)) for o in outs]
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()


def common_window(res, min_frac=0.5):
    """Every pod's throughput over the window in which all of them run: from the latest
    start to the earliest last completed step. Each pod measures its own window, and these
    differ at the ends by up to the steps it has queued (4 between waits: most of a second
    for a 16-pod share of ResNet-50); a pod still running after the others stop has the GPU
    to itself and looks faster, the others slower. A step counts in proportion to the part
    of (previous completion, its completion] inside the window. Returns (per-pod items/s,
    window seconds), or None when the window is shorter than ``min_frac`` of the pods'
    median run (the own-window rates stand then)."""
    if not res or any(not r.get("step_done") for r in res):
        return None
    w0 = max(r["t0"] for r in res)
    w1 = min(r["step_done"][-1] for r in res)
    runs = sorted(r["t1"] - r["t0"] for r in res)
    if w1 - w0 < min_frac * runs[len(runs) // 2]:
        return None
    rates = []
    for r in res:
        items, prev = 0.0, r["t0"]
        for done in r["step_done"]:
            lo, hi = max(prev, w0), min(done, w1)
            if hi > lo and done > prev:
                items += r["items_per_step"] * (hi - lo) / (done - prev)
            prev = done
        rates.append(items / (w1 - w0))
    return rates, w1 - w0


def miopen_env(mode, root, i):
    """MIOpen find-db / kernel cache of sweep pod ``i`` (``--sweep-find-db``)."""
    if mode == "home":
        return None
    import shutil
    db, cache = os.path.join(root, f"pod{i}", "db"), os.path.join(root, f"pod{i}", "cache")
    home = os.path.expanduser("~")
    for src, dst in ((os.path.join(home, ".config", "miopen"), db), (os.path.join(home, ".cache", "miopen"), cache)):
        if mode == "per-pod" and os.path.isdir(src):
            shutil.copytree(src, dst, dirs_exist_ok=True)
        os.makedirs(dst, exist_ok=True)
    return {"MIOPEN_USER_DB_PATH": db, "MIOPEN_CUSTOM_CACHE_DIR": cache}


def sweep(args, backend, uuid, tenants):
    import shutil
    rows, skipped = [], []
    end = T_START + args.time_budget
    root = tempfile.mkdtemp(prefix="bench-miopen-")
    try:
        rows, skipped = _sweep_points(args, backend, uuid, tenants, end, root)
    finally:
        shutil.rmtree(root, ignore_errors=True)
    base = next((r["aggregate"] for r in rows if r["tenants"] == 1), None)
    best = 0
    for r in rows:
        if not base:
            break
        r["aggregate_vs_one"] = round(r["aggregate"] / base, 3)
        r["min_tenant_vs_entitlement"] = round(min(r["per_tenant"]) / (base / r["tenants"]), 3)
        r["ok"] = r["aggregate_vs_one"] >= SWEEP_MIN_AGGREGATE and r["min_tenant_vs_entitlement"] >= SWEEP_MIN_TENANT
        if r["ok"]:
            best = max(best, r["tenants"])
    return rows + skipped, best


def _sweep_points(args, backend, uuid, tenants, end, root):
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    rows, skipped = [], []
    last = None  # (pods, seconds) of the last measured point with several pods
    for n in tenants:
        t_point = now()
        # Start-up dominates a point and grows about linearly with the pods (each warms up,
        # MIOpen find included, on its share of the GPU): skip what would not finish.
        est = last[1] * n / last[0] if last else 20.0 + 8.0 * n
        if t_point + est > end:
            skipped.append({"tenants": n, "skipped": f"time budget: ~{est:.0f} s needed, {end - t_point:.0f} s left"})
            print(f"[bench] sweep {n} tenants skipped ({skipped[-1]['skipped']})", file=sys.stderr, flush=True)
            continue
        try:
            with NodeHarness(backend, device_split_count=n, cu_mode=args.cu_mode, **ledger_kw(args)) as node:
                ids = node.vgpu_ids(uuid)[:n]
                # The lone pod runs on this process's own find-db (the native run filled it);
                # with several, each pod gets its own (--sweep-find-db).
                extra = dict(kv.split("=", 1) for kv in args.sweep_pod_env)
                pods = [pod_env(node, [i], {**(miopen_env(args.sweep_find_db if n > 1 else "home", root,
                                                          k + 100 * n + 1000 * len(rows)) or {}), **extra})
                        for k, i in enumerate(ids)]
                res = run_concurrent(args, [e for e, _ in pods], f"sweep{n}",
                                     deadline=end - args.sweep_seconds - 15.0)
                c0 = pods[0][1]
        except OutOfTime as e:
            skipped.append({"tenants": n, "skipped": f"time budget: {e}"})
            print(f"[bench] sweep {n} tenants abandoned ({e})", file=sys.stderr, flush=True)
            continue
        if n > 1:
            last = (n, now() - t_point)
        own = [r["items_per_step"] * r["steps"] / (r["t1"] - r["t0"]) for r in res]
        span = max(r["t1"] for r in res) - min(r["t0"] for r in res)
        agg_span = sum(r["items_per_step"] * r["steps"] for r in res) / span
        cw = common_window(res)
        tput, agg = (cw[0], sum(cw[0])) if cw else (own, agg_span)
        rows.append({"tenants": n, "aggregate": round(agg, 2), "per_tenant": [round(t, 2) for t in tput],
                     "window": f"common {cw[1]:.2f} s" if cw else "own",
                     "per_tenant_own_window": [round(t, 2) for t in own], "aggregate_span": round(agg_span, 2),
                     "cpus_busy": round(sum(r.get("cpu_s", 0.0) for r in res) / span, 2),
                     "pod_wait": res[0].get("wait"),
                     # per pod: GPU time charged by its limiter over its window (% of wall), and the
                     # enforcement at the end of the window
                     "granted_pct": [r.get("granted_pct") for r in res],
                     "throttled_pct": [r.get("throttled_pct") for r in res],
                     "region_procs": [r.get("region_procs") for r in res],
                     "cu_mode_end": sorted({str(r.get("cu_mode_end")) for r in res}),
                     "cu_limit_pct": int(c0.get("VGPU_DEVICE_CU_LIMIT_0", "0") or 0),
                     "cu_mode": c0.get("VGPU_CU_MODE"), "quota_mib": int(c0["VGPU_DEVICE_MEMORY_LIMIT_0"].rstrip("m"))})
        print(f"[bench] sweep {n} tenants: aggregate {agg:.1f}, per tenant {min(tput):.1f}..{max(tput):.1f} "
              f"({now() - t_point:.0f} s)", file=sys.stderr, flush=True)
    return rows, skipped


def node_point(args, backend, uuid, world, rank, port):
    """BASELINE config 5 on the GPUs of this job: every GPU split ``--split`` ways with all of
    its vGPUs busy at once (8 GPUs x 4 = 32 vGPUs on a full node). Each rank runs the pods of
    its own GPU (one plugin per rank, as in the other modes); a gloo barrier between the
    ranks' parents releases every pod of the node in the same window. Every rank reaches the
    barrier even when its pods fail, so a failure is reported, never a hang. Returns the
    per-rank records on rank 0 (None elsewhere)."""
    import datetime

    import torch.distributed as dist
    from amdvgpu.plugin.kubelet_stub import NodeHarness
    if world > 1:
        # Under torchrun the rank would otherwise look for the agent's store on this port
        # instead of rank 0 serving it (the workers drop the variable for the same reason).
        os.environ.pop("TORCHELASTIC_USE_AGENT_STORE", None)
        dist.init_process_group("gloo", init_method=f"tcp://{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{port}",
                                rank=rank, world_size=world, timeout=datetime.timedelta(seconds=600))
    passed = [False]

    def gate():
        passed[0] = True  # attempted: a barrier that timed out is not entered twice
        if world > 1:
            dist.barrier()

    t_point = now()
    try:
        with NodeHarness(backend, device_split_count=args.split, cu_mode=args.cu_mode, **ledger_kw(args)) as node:
            ids = node.vgpu_ids(uuid)[:args.split]
            envs = [pod_env(node, [i])[0] for i in ids]
            res = run_concurrent(args, envs, "node", deadline=T_START + args.time_budget - args.sweep_seconds - 15.0,
                                 before_go=gate)
        own = [round(r["items_per_step"] * r["steps"] / (r["t1"] - r["t0"]), 2) for r in res]
        cw = common_window(res)
        mine = {"ok": True, "uuid": uuid, "pods": len(res),
                "per_pod": [round(t, 2) for t in cw[0]] if cw else own, "per_pod_own_window": own,
                "window": f"common {cw[1]:.2f} s" if cw else "own",
                "seconds": round(now() - t_point, 1)}
    except (Exception, SystemExit) as e:  # noqa: BLE001 - reported in the line, never a hang
        if not passed[0] and world > 1:
            dist.barrier()
        mine = {"ok": False, "uuid": uuid, "error": repr(e)[:300]}
    print(f"[bench] node point (rank {rank}): {mine}", file=sys.stderr, flush=True)
    if world == 1:
        return [mine]
    out = [None] * world
    dist.all_gather_object(out, mine)
    dist.destroy_process_group()
    return out if rank == 0 else None


def node_summary(records, split, native_per_gpu):
    """The node point's line entry: aggregate over every vGPU of the job and the slowest
    pod against its 1/split entitlement of a native GPU."""
    ok = [r for r in records if r.get("ok")]
    s = {"pods_per_gpu": split, "vgpus": split * len(records), "gpus_measured": len(ok),
         "failures": [r for r in records if not r.get("ok")]}
    if not ok:
        return s
    pods = [t for r in ok for t in r["per_pod"]]
    s["aggregate"] = round(sum(pods), 2)
    s["per_pod_min"], s["per_pod_max"] = min(pods), max(pods)
    if native_per_gpu:
        s["aggregate_vs_native"] = round(s["aggregate"] / (native_per_gpu * len(ok)), 3)
        s["min_pod_vs_entitlement"] = round(min(pods) / (native_per_gpu / split), 3)
    return s


def make_backend(cpu, world):
    """The rank's device inventory: the node's GPUs from KFD sysfs (no GPU context), or in
    the CPU rehearsal a fake node of WORLD_SIZE GPUs (``VGPU_BENCH_FAKE_GPUS`` overrides
    the count, so a too-small node can be rehearsed)."""
    from amdvgpu.plugin.devices import FakeBackend, SysfsBackend
    if cpu:
        return FakeBackend(n=int(os.environ.get("VGPU_BENCH_FAKE_GPUS", 0) or max(world, 1)))
    return SysfsBackend()


def visible_devices(backend, cpu):
    """The GPUs this job may use, in KFD order: every GPU whose render node this process can
    open (a container sees every GPU's sysfs but only its own device nodes), narrowed by
    ROCR_VISIBLE_DEVICES / HIP_VISIBLE_DEVICES (indices or UUIDs) when set. Reads sysfs
    and device-node permissions only; never opens a GPU context."""
    devs = backend.devices()
    if cpu:
        return devs
    usable = [d for d in devs if d.render_minor < 0 or os.access(f"/dev/dri/renderD{d.render_minor}", os.R_OK | os.W_OK)]
    devs = usable or devs
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES"):
        sel = os.environ.get(var, "").strip()
        if not sel:
            continue  # unset or empty: no narrowing
        picked = []
        for tok in (t.strip() for t in sel.split(",") if t.strip()):
            if tok.isdigit():
                if int(tok) < len(devs):
                    picked.append(devs[int(tok)])
            else:
                picked += [d for d in devs if d.uuid == tok]
        devs = picked
    return devs


def free_port_range(span=32):
    """A free port P on 127.0.0.1 whose next ``span`` ports are free as well: the ranks'
    worker process groups sit on MASTER_PORT+1, +2, ... (one per mode and probe)."""
    import socket
    for _ in range(200):
        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        p = s.getsockname()[1]
        s.close()
        if p + span >= 65536:
            continue
        ok = True
        for q in range(p + 1, p + span + 1):
            t = socket.socket()
            try:
                t.bind(("127.0.0.1", q))
            except OSError:
                ok = False
            finally:
                t.close()
            if not ok:
                break
        if ok:
            return p
    raise SystemExit("bench: no free port range on 127.0.0.1 for the ranks")


def self_launch(args, argv):
    """``--gpus N > 1`` without a launcher: this process (which never touches a GPU) starts
    the N ranks itself under torch.distributed.run - one rank per GPU, rendezvous on
    127.0.0.1 - and exits with their exit code; rank 0 prints the line. A job asking for
    more GPUs than are visible is refused (non-zero exit), never measured on fewer."""
    devices = visible_devices(make_backend(args.cpu_rehearsal, args.gpus), args.cpu_rehearsal)
    if args.gpus > len(devices):
        print(f"bench: --gpus {args.gpus} but only {len(devices)} GPU(s) visible to this job "
              f"({', '.join(d.uuid for d in devices) or 'none'}); refusing to report a smaller job",
              file=sys.stderr, flush=True)
        return 2
    port = int(os.environ.get("MASTER_PORT", 0) or 0) or free_port_range()
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + list(argv)
    env = dict(os.environ, MASTER_ADDR="127.0.0.1")
    print(f"[bench] launching {args.gpus} ranks (torch.distributed.run, master 127.0.0.1:{port})",
          file=sys.stderr, flush=True)
    return subprocess.call(cmd, env=env)


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse(argv)
    if args.worker:
        return worker(args)
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        return self_launch(args, argv)
    from amdvgpu.models.aibench import get_case
    from amdvgpu.plugin.kubelet_stub import NodeHarness

    world = int(os.environ.get("WORLD_SIZE", 1))
    rank = int(os.environ.get("RANK", 0))
    local = int(os.environ.get("LOCAL_RANK", 0))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    cpu = args.cpu_rehearsal
    backend = make_backend(cpu, world)
    devices = visible_devices(backend, cpu)
    if world > len(devices):
        # every rank refuses alike, so none waits on a rendezvous the others never reach
        raise SystemExit(f"bench: WORLD_SIZE {world} but only {len(devices)} GPU(s) visible to this job")
    uuid = devices[local].uuid
    base_port = int(os.environ.get("MASTER_PORT", 29500))
    modes = [m for m in args.modes.split(",") if m]
    results, contracts, applied = {}, {}, {}
    port = base_port + 1
    for mode in modes:
        if mode == "native":
            results[mode] = run_one(args, mode, native_env(uuid, cpu), port)
        else:
            # quota: the split's memory quota with the compute share lifted by the plugin itself
            # (cores scaling = split -> 100 %: no CU limit in the contract), so the number is the
            # interception cost alone. parity: the reference's contract; --host-memory-fraction 0
            # as the reference has no node bound on the host memory its spill may pin.
            split, scaling, cores, extra_cfg = {
                "vgpu": (args.split, 1.0, 1.0, {}), "quota": (args.split, 1.0, float(args.split), {}),
                "parity": (2, 1.8, 1.0, {"host_memory_fraction": 0.0})}[mode]
            with NodeHarness(backend, device_split_count=split, device_memory_scaling=scaling, device_cores_scaling=cores,
                             **ledger_kw(args), **extra_cfg, cu_mode=args.cu_mode) as node:
                env, contracts[mode] = pod_env(node, node.vgpu_ids(uuid)[:1], None)
                applied[mode] = {k: env.get(k) for k in ("ROCR_VISIBLE_DEVICES", "VGPU_SHARED_CACHE", "VGPU_ALLOWLIST",
                                                         "VGPU_LOCK_FILE", "VGPU_DEVICE_MAP")}
                applied[mode]["node_dir"] = node.dir
                results[mode] = run_one(args, mode, env, port)
        port += 1
    if cpu and os.environ.get("VGPU_BENCH_CONTRACT_DIR"):
        # Rehearsal evidence: every rank's pods, as the container runtime would see them
        # (tests/test_bench_contract.py checks that the ranks' node harnesses never collide).
        with open(os.path.join(os.environ["VGPU_BENCH_CONTRACT_DIR"], f"rank{rank}.json"), "w") as f:
            json.dump({"rank": rank, "local_rank": local, "uuid": uuid, "pods": applied}, f)
    rccl = None
    if world > 1 and args.rccl_probe:
        # an all-reduce between vGPUs of different GPUs must run at the native
        # xGMI bandwidth. Same ranks, same size: without the shim, then inside the pods.
        rccl = {"native": probe_rccl(args, native_env(uuid, cpu), port)}
        port += 1
        with NodeHarness(backend, device_split_count=args.split, cu_mode=args.cu_mode, **ledger_kw(args)) as node:
            env, _ = pod_env(node, node.vgpu_ids(uuid)[:1])
            rccl["vgpu"] = probe_rccl(args, env, port)
        port += 1
        if rank == 0 and all(isinstance(v, dict) and (v.get("busbw_GBps") or 0) > 0 for v in rccl.values()):
            rccl["vgpu_vs_native_busbw"] = round(rccl["vgpu"]["busbw_GBps"] / rccl["native"]["busbw_GBps"], 3)
    node = None
    if args.node == "on" or (args.node == "auto" and world > 1):
        node = node_point(args, backend, uuid, world, rank, port)
        port += 1
    do_sweep = args.sweep == "on" or (args.sweep == "auto" and world == 1 and not cpu)
    sweep_rows, max_vgpus = ([], None)
    if do_sweep:
        sweep_rows, max_vgpus = sweep(args, backend, uuid, [int(x) for x in args.sweep_tenants.split(",")])
    if rank != 0:
        return 0

    case = get_case(args.case)
    head_mode = "vgpu" if "vgpu" in results else modes[-1]
    head = results[head_mode]
    ms = head["ms_per_step"]
    value = world * head["items_per_step"] * 1000.0 / ms
    c = contracts.get("vgpu", {})
    cu_pct = int(c.get("VGPU_DEVICE_CU_LIMIT_0", "0") or 0)
    line = {
        "metric": METRIC if args.case == "resnet50-inf" else f"ai-benchmark {case.model} "
                  f"{'training' if case.train else 'inference'} throughput inside a vGPU ({case.unit})",
        "value": round(value, 3),
        "unit": case.unit,
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": round(value / (case.baseline_vgpu * world), 3) if case.baseline_vgpu else None,
        "dtype": args.dtype,
        "data": "synthetic (random-init weights, random inputs)",
        "config": {
            "model": case.model, "test": case.test_id, "mode": "training" if case.train else "inference",
            "global_batch": case.batch * world, "per_gpu_batch": case.batch,
            "input_shape": list(case.input_shape), "seq_len": None,
            "parallelism": f"dp{world} (one independent split-{args.split} vGPU pod per GPU)",
            "workload": "stock PyTorch-ROCm (MIOpen/hipBLASLt), no custom kernels",
            "vgpu": {"split": args.split, "source": "Allocate response of the plugin (sysfs backend, stub kubelet)",
                     "envs": {k: v for k, v in sorted(c.items()) if k.startswith("VGPU_") and k != "VGPU_SHARED_CACHE"},
                     "quota_bytes": int(c.get("VGPU_DEVICE_MEMORY_LIMIT_0", "0").rstrip("m") or 0) << 20,
                     "cu_limit_pct": cu_pct, "cu_mode": c.get("VGPU_CU_MODE"),
                     "node_ledger": bool(args.ledger if args.ledger is not None else plugin_default_ledger())},
        },
    }
    nat = results.get("native", {}).get("ms_per_step") if results.get("native") else None
    if nat:
        line["ms_per_batch_native"] = round(nat, 4)
        if "vgpu" in results:
            line["ms_per_batch_vgpu"] = round(ms, 4)
            share = cu_pct / 100.0 if 0 < cu_pct < 100 else 1.0
            # The pod's throughput over what its compute share entitles it to (native x share).
            line["entitlement_ratio"] = round(nat / (ms * share), 3)
            line["overhead_pct_vs_native_x_share"] = round((ms * share - nat) / nat * 100.0, 3)
            for k in ("limiter_granted_pct", "gpu_ms_charged_per_step", "effective_cu_mode", "crowd"):
                if k in results["vgpu"]:
                    line[k] = results["vgpu"][k]
        if "quota" in results:
            q = results["quota"]["ms_per_step"]
            line["ms_per_batch_quota_only"] = round(q, 4)
            line["overhead_pct_quota_only"] = round((q - nat) / nat * 100.0, 3)
        if "parity" in results:
            p = results["parity"]["ms_per_step"]
            pc = contracts["parity"]
            pct = int(pc.get("VGPU_DEVICE_CU_LIMIT_0", "0") or 0)
            line["parity_split2_mem1.8"] = {
                "ms_per_batch": round(p, 4),
                "throughput": round(world * results["parity"]["items_per_step"] * 1000 / p, 3),
                "cu_limit_pct": pct, "cu_mode": pc.get("VGPU_CU_MODE"),
                "oversubscribe": pc.get("VGPU_OVERSUBSCRIBE") == "true",
                "quota_bytes": int(pc["VGPU_DEVICE_MEMORY_LIMIT_0"].rstrip("m")) << 20,
                "hbm_limit_bytes": int(pc.get("VGPU_DEVICE_HBM_LIMIT_0", "0").rstrip("m") or 0) << 20,
                "entitlement_ratio": round(nat / (p * (pct / 100.0 if 0 < pct < 100 else 1.0)), 3)}
        # Reference's own vGPU overhead on this case (2xV100, BASELINE.md "Derived ms/batch").
        line["reference_overhead_pct"] = round((case.baseline_native / case.baseline_vgpu - 1) * 100.0, 2)
    if rccl is not None:
        line["rccl_allreduce_between_pods"] = rccl
    native_per_gpu = results["native"]["items_per_step"] * 1000.0 / nat if nat else None
    if node is not None:
        line["node"] = node_summary(node, args.split, native_per_gpu)
    elif do_sweep:
        # Single GPU: the sweep's point with --split pods is the node point of a 1-GPU job.
        row = next((r for r in sweep_rows if r.get("tenants") == args.split and "per_tenant" in r), None)
        if row:
            line["node"] = node_summary([{"ok": True, "per_pod": row["per_tenant"]}], args.split, native_per_gpu)
    if do_sweep:
        line["max_vgpus_per_gpu"] = max_vgpus
        line["max_vgpus_criterion"] = (f"largest N with aggregate >= {SWEEP_MIN_AGGREGATE}x one whole-GPU pod and "
                                       f"slowest pod >= {SWEEP_MIN_TENANT}x its 1/N entitlement "
                                       f"(tested N = {','.join(str(r['tenants']) for r in sweep_rows if 'skipped' not in r)})")
        line["sweep"] = sweep_rows
        line["sweep_find_db"] = args.sweep_find_db
    line["baseline_vgpu_v100"] = case.baseline_vgpu
    out = json.dumps(line)
    print(out, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(out + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
