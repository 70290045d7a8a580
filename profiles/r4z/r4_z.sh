#!/bin/bash
# Round-4 GPU study (profiles/r4z): is the 16-pod point CPU-bound on the box's 16-CPU quota?
# bench.py's sweep (ledger default, per-pod find-db copied after the native run's find) with
# every pod's CPU seconds in its window, in MIOpen immediate mode (the default) and in find
# mode (PyTorch caches each convolution's algorithm: no per-call MIOpen solution query).
out=${1:-gpurun_out/r4z}
mkdir -p "$out"
for at in 0 1; do
  timeout -k 10 420 python -u bench.py --modes native --sweep on --sweep-tenants 1,8,12,16 --sweep-autotune $at \
    --rccl-probe 0 --time-budget 380 --json-out "$out/at$at.json" > "$out/at$at.log" 2>&1
  rc=$?
  echo "bench_rc=$rc" >> "$out/at$at.log"
  [ $rc -eq 0 ] || exit $rc
done
