#!/bin/bash
# Round-4 GPU study (profiles/r4za): which threads of a GPU-bound ResNet-50 pod use its CPU
# time, natively and in a quota vGPU, for the bench's blocking wait every 4 steps, torch's
# default (spinning) synchronize, and a blocking wait after every step.
out=${1:-gpurun_out/r4za}
mkdir -p "$out"
for s in block spin every; do
  timeout -k 10 200 python -u tools/probe/cpu_probe.py --sync $s --modes native,vgpu >> "$out/cpu.log" 2>&1
  rc=$?
  echo "sync=$s rc=$rc" >> "$out/cpu.log"
  [ $rc -eq 0 ] || exit $rc
done
