#!/usr/bin/env python3
"""Hardware-counter evidence of the spatial CU limit (north star: "occupancy shown with
rocprof counters").

Runs one workload as a "container" under a vGPU contract (or natively) so that
``rocprofv3 --pmc`` can count, per dispatch, how many CU-cycles were busy:

* ``spin``    single-wave workgroups, 8 per CU of the whole chip, each spinning a fixed
              time: a kernel that would keep every CU busy if it could reach them.
* ``resnet``  ResNet-V2-50 inference (ai-benchmark 1.1 shape, stock fp32 PyTorch), a real
              workload: its MIOpen / hipBLASLt kernels size their grids for the whole GPU.

The parent never touches the GPU; it starts the worker with the contract applied
(``shim/launcher.py``), so under ``rocprofv3 -- python3 benchmarks/cu_occupancy.py ...``
the profiler's preload and the shim's preload both reach the worker.

    rocprofv3 --pmc SIMD_UTILIZATION SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE \\
        --kernel-trace --output-format csv -d OUT -o native -- \\
        python3 benchmarks/cu_occupancy.py --cu-limit 0
    python tools/pmc_summary.py OUT/**/native_counter_collection.csv ...
"""
import argparse
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def worker(a):
    import torch
    from amdvgpu.ops import spin
    if "spin" in a.workload:
        for _ in range(a.iters):
            spin(256 * 8, a.spin_us)
        torch.cuda.synchronize()
    if "resnet" in a.workload:
        from amdvgpu.models.aibench import Runner, get_case
        torch.backends.cudnn.benchmark = False
        r = Runner(get_case("resnet50-inf"), "cuda")  # stock fp32 tenant
        for _ in range(a.iters):
            r.step()
        torch.cuda.synchronize()
    free, total = torch.cuda.mem_get_info()
    print(f"worker cu_limit={a.cu_limit} mem_total={total}", flush=True)
    return 0


def main(argv=None):
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--cu-limit", type=int, default=0, help="vGPU CU share %% (0 = native, no shim)")
    ap.add_argument("--cu-mode", default="spatial", help="the vGPU's VGPU_CU_MODE (spatial: CU mask; temporal: "
                    "GPU-time limiter on all CUs)")
    ap.add_argument("--workload", default="spin,resnet")
    ap.add_argument("--iters", type=int, default=3)
    ap.add_argument("--spin-us", type=int, default=200)
    ap.add_argument("--worker", action="store_true")
    a = ap.parse_args(argv)
    if a.worker:
        return worker(a)
    from amdvgpu.shim.launcher import apply_contract, cleanup_region, vgpu_env
    cmd = [sys.executable, os.path.abspath(__file__), "--worker", "--cu-limit", str(a.cu_limit),
           "--workload", a.workload, "--iters", str(a.iters), "--spin-us", str(a.spin_us)]
    if a.cu_limit <= 0:
        return subprocess.call(cmd)
    contract = vgpu_env(mem_limit=72 << 30, cu_limit=a.cu_limit, cu_mode=a.cu_mode)
    try:
        return subprocess.call(cmd, env=apply_contract(contract))
    finally:
        cleanup_region(contract)


if __name__ == "__main__":
    sys.exit(main())
