#!/bin/bash
# Round-4 GPU study (profiles/r4v): where the PyTorch-level per-op cost under the shim comes
# from. (1) DeepLab training b=1 in the suite's interception-only pod with VGPU_STATS=1: how
# many launches leave the gate's fast path. (2) The PyTorch per-op loop natively, in a vGPU,
# with the launch gates made pass-throughs and with the dlsym routing off, 6 repeats.
out=${1:-gpurun_out/r4v}
mkdir -p "$out"
VGPU_STATS=1 timeout -k 10 300 python -u benchmarks/aibench_suite.py --cases deeplab-train --modes native,vgpu \
  --repeats 2 --steps 50 --vdm 0 --json-out "$out/census.json" > "$out/census.log" 2>&1
rc=$?
echo "census_rc=$rc" >> "$out/census.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 400 python -u benchmarks/hook_overhead.py --iters 20000 --repeats 6 \
  --modes native,vgpu,vgpu-nogate,vgpu-nodlsym --json-out "$out/hooks.json" --md-out "$out/hooks.md" \
  > "$out/hooks.log" 2>&1
echo "hooks_rc=$?" >> "$out/hooks.log"
