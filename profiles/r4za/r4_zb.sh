#!/bin/bash
# Round-4 GPU study (profiles/r4za, part 2): the HIP runtime's host-wait settings and a
# GPU-bound pod's CPU time (native, blocking wait every 4 steps).
out=${1:-gpurun_out/r4za}
mkdir -p "$out"
for e in ROC_ACTIVE_WAIT_TIMEOUT=0 AMD_DIRECT_DISPATCH=0 ROC_CPU_WAIT_FOR_SIGNAL=1 HIP_LAUNCH_BLOCKING=0; do
  timeout -k 10 120 python -u tools/probe/cpu_probe.py --sync block --modes native --extra-env $e >> "$out/env.log" 2>&1
  rc=$?
  echo "env=$e rc=$rc" >> "$out/env.log"
  [ $rc -eq 0 ] || exit $rc
done
