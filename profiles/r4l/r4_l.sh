#!/bin/bash
# Round-4 GPU study (profiles/r4l): 16-pod start-up when the pods skip MIOpen's per-process
# find (immediate mode; --sweep-autotune 0, the lone pod too), and the sweep's per-pod
# find-db copies with the default autotuning, both through bench.py's sweep.
out=${1:-gpurun_out/r4l}
mkdir -p "$out"
timeout -k 10 420 python -u bench.py --modes native --sweep on --sweep-tenants 1,16 --sweep-seconds 8 \
  --sweep-autotune 0 --time-budget 400 --json-out "$out/noauto.json" > "$out/noauto.log" 2>&1 || exit $?
timeout -k 10 420 python -u bench.py --modes native --sweep on --sweep-tenants 1,16 --sweep-seconds 8 \
  --time-budget 400 --json-out "$out/perpod.json" > "$out/perpod.log" 2>&1 || exit $?
