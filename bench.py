#!/usr/bin/env python3
"""Headline benchmark: ai-benchmark ResNet-V2-50 inference (test 1.1) inside a vGPU.

Mirrors the reference's published measurement (README.md:38-72): the same
workload run natively and inside a vGPU container, reporting the vGPU's throughput and
its ms/batch overhead versus native. Here the vGPU is a 4-way split of one MI355X
(72 GiB HBM quota, BASELINE.json config 2) enforced by the in-tree interception shim
(libvgpu_hip.so), applied to the worker exactly as the container runtime would apply the
plugin's Allocate response (env contract + preload).

Process layout (one rank per GPU under torch.distributed.run): the rank process never
touches the GPU; it starts one worker child per mode (native, then vgpu), each of which
initialises RCCL, runs W untimed warmup steps, then times exactly K steps bracketed by
barrier + synchronize on both sides, and reduces the MAX step time over ranks. Rank 0
prints one JSON line. ``value`` is the whole-job vGPU throughput (sum over GPUs).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--case resnet50-inf]
                    [--modes native,vgpu] [--split 4] [--cu-limit 0]
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, REPO)

MI355X_HBM_BYTES = 309220868096  # 288 GiB as reported by ROCr on the box (gpurun_out probe)
METRIC = "ai-benchmark ResNet-V2-50 inference throughput inside a vGPU (images/s); ms/batch overhead vs native"


def parse(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--case", default="resnet50-inf")
    ap.add_argument("--modes", default="native,vgpu")
    ap.add_argument("--split", type=int, default=4, help="vGPUs per physical GPU (quota = HBM / split)")
    ap.add_argument("--memory-scaling", type=float, default=1.0)
    ap.add_argument("--cu-limit", type=int, default=0, help="CU share %% of the vGPU (0 = quota only)")
    ap.add_argument("--cu-mode", default="spatial", choices=["spatial", "temporal", "both", "off"])
    ap.add_argument("--dtype", default="bf16", choices=["bf16", "fp32"])
    ap.add_argument("--no-fuse", action="store_true", help="eager PyTorch epilogues (no fused HIP BN+ReLU)")
    ap.add_argument("--tune", type=int, default=1, choices=[0, 1],
                    help="MIOpen find-mode conv autotuning during warmup (torch.backends.cudnn.benchmark); "
                         "the reference's TensorFlow autotunes convolutions too")
    ap.add_argument("--json-out", default=None, help="also write the result line to this file")
    # worker-only
    ap.add_argument("--worker", action="store_true", help=argparse.SUPPRESS)
    ap.add_argument("--mode", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--result-file", default=None, help=argparse.SUPPRESS)
    ap.add_argument("--port", type=int, default=0, help=argparse.SUPPRESS)
    # CPU rehearsal of the multi-rank orchestration (gloo, tiny batch); not a measurement
    ap.add_argument("--cpu-rehearsal", action="store_true", help=argparse.SUPPRESS)
    return ap.parse_args(argv)


# ----------------------------------------------------------------------------- worker


def worker(args):
    import torch
    import torch.distributed as dist

    from amdvgpu.models.aibench import Runner, get_case

    rank = int(os.environ.get("RANK", 0))
    world = int(os.environ.get("WORLD_SIZE", 1))
    local = int(os.environ.get("LOCAL_RANK", 0))
    cpu = args.cpu_rehearsal
    if cpu:
        device = torch.device("cpu")
    else:
        torch.cuda.set_device(local)
        device = torch.device("cuda", local)
    if world > 1:
        init = f"tcp://{os.environ.get('MASTER_ADDR', '127.0.0.1')}:{args.port}"
        if cpu:
            dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
        else:
            dist.init_process_group("nccl", init_method=init, rank=rank, world_size=world, device_id=device)

    sync = (lambda: None) if cpu else (lambda: torch.cuda.synchronize(device))
    free0, total = torch.cuda.mem_get_info(device) if not cpu else (0, 0)
    if args.mode == "vgpu" and not cpu:
        quota = int(os.environ["VGPU_DEVICE_MEMORY_LIMIT"].rstrip("m")) << 20
        if total != min(quota, MI355X_HBM_BYTES) and not os.environ.get("VGPU_OVERSUBSCRIBE"):
            raise SystemExit(f"vGPU shim not in effect: mem_get_info total {total} != quota {quota}")

    torch.backends.cudnn.benchmark = bool(args.tune)
    case = get_case(args.case)
    dtype = torch.bfloat16 if args.dtype == "bf16" else torch.float32
    if cpu:
        runner = Runner(case, device, dtype=torch.float32, batch=2, channels_last=False, fuse=False)
        runner.x = runner.x[..., :64, :64].contiguous() if runner.x.dim() == 4 else runner.x[:, :16].contiguous()
    else:
        runner = Runner(case, device, dtype=dtype, fuse=not args.no_fuse)
    for _ in range(args.warmup):
        runner.step()
    sync()

    def barrier():
        if world > 1:
            dist.barrier(device_ids=[local]) if not cpu else dist.barrier()
        sync()

    barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        runner.step()
    sync()
    barrier()
    dt = time.perf_counter() - t0
    ms = torch.tensor([dt * 1000.0 / args.steps], dtype=torch.float64, device=device)
    if world > 1:
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    res = {
        "mode": args.mode, "ms_per_step": ms.item(), "items_per_step": runner.items_per_step,
        "mem_total": total, "world": world,
        "peak_allocated": torch.cuda.max_memory_allocated(device) if not cpu else 0,
    }
    if rank == 0 and args.result_file:
        with open(args.result_file, "w") as f:
            json.dump(res, f)
    if world > 1:
        barrier()
        dist.destroy_process_group()
    return 0


# ----------------------------------------------------------------------------- parent


def run_mode(args, mode, port):
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env

    rank = int(os.environ.get("RANK", 0))
    fd, result = tempfile.mkstemp(prefix=f"bench-{mode}-", suffix=".json")
    os.close(fd)
    cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--mode", mode, "--result-file", result,
           "--port", str(port), "--case", args.case, "--steps", str(args.steps), "--warmup", str(args.warmup),
           "--dtype", args.dtype, "--tune", str(args.tune)] + (["--no-fuse"] if args.no_fuse else []) + \
        (["--cpu-rehearsal"] if args.cpu_rehearsal else [])
    contract = {}
    if mode == "vgpu":
        quota = int(MI355X_HBM_BYTES * args.memory_scaling / args.split)
        contract = vgpu_env(mem_limit=quota, cu_limit=args.cu_limit or None, cu_mode=args.cu_mode,
                            oversubscribe=args.memory_scaling > 1,
                            shared_cache=os.path.join(tempfile.gettempdir(), f"vgpu-bench-{os.getpid()}-{rank}.cache"))
        env = apply_contract(contract)
    else:
        env = dict(os.environ)
    # The worker hosts its own rendezvous store on `port` (rank 0); under
    # torch.distributed.run the agent's store flag would make every worker a client of a
    # store that does not exist on that port.
    env.pop("TORCHELASTIC_USE_AGENT_STORE", None)
    try:
        rc = subprocess.call(cmd, env=env)
        if rc != 0:
            raise SystemExit(f"bench worker ({mode}) failed with exit code {rc}")
        if rank != 0:
            return None
        with open(result) as f:
            return json.load(f)
    finally:
        os.unlink(result)
        if contract:
            cleanup_region(contract)


def main(argv=None):
    args = parse(argv)
    if args.worker:
        return worker(args)
    world = int(os.environ.get("WORLD_SIZE", 1))
    if world != args.gpus:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE={world}; using WORLD_SIZE", file=sys.stderr)
    base_port = int(os.environ.get("MASTER_PORT", 29500))
    modes = [m for m in args.modes.split(",") if m]
    results = {}
    for i, mode in enumerate(modes):
        results[mode] = run_mode(args, mode, base_port + 1 + i)
    if int(os.environ.get("RANK", 0)) != 0:
        return 0

    from amdvgpu.models.aibench import get_case
    case = get_case(args.case)
    head = results.get("vgpu") or results[modes[-1]]
    ms = head["ms_per_step"]
    value = world * head["items_per_step"] * 1000.0 / ms
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
            "parallelism": f"dp{world} (one independent vGPU replica per GPU)",
            "fused_epilogues": not args.no_fuse,
            "conv_autotune": bool(args.tune),
            "vgpu": {"split": args.split, "quota_bytes": int(MI355X_HBM_BYTES * args.memory_scaling / args.split),
                     # CU-mask granularity is one CU per XCD (8 CUs): 256 / 8 disjoint slices
                     "max_vgpus_per_gpu_spatial": 32,
                     "cu_limit_pct": args.cu_limit, "cu_mode": args.cu_mode,
                     "memory_scaling": args.memory_scaling},
        },
    }
    if "native" in results and "vgpu" in results:
        nat = results["native"]["ms_per_step"]
        line["ms_per_batch_native"] = round(nat, 4)
        line["ms_per_batch_vgpu"] = round(ms, 4)
        line["overhead_pct_vs_native"] = round((ms - nat) / nat * 100.0, 3)
        # Reference's own vGPU overhead on this case (2xV100, BASELINE.md "Derived ms/batch").
        line["reference_overhead_pct"] = round((case.baseline_native / case.baseline_vgpu - 1) * 100.0, 2)
    line["baseline_vgpu_v100"] = case.baseline_vgpu
    out = json.dumps(line)
    print(out, flush=True)
    if args.json_out:
        with open(args.json_out, "w") as f:
            f.write(out + "\n")
    return 0


if __name__ == "__main__":
    sys.exit(main())
