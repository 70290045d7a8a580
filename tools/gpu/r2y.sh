#!/bin/bash
# Round 2y: slice CU count in auto mode — test, then the full default bench.
out=gpurun_out/r2y; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 300 python -u -m pytest tests/test_gpu_limits.py -k "cu_count" -v -s --timeout 200 --timeout-method thread
step bench 900 python -u bench.py
