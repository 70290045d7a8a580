#!/bin/bash
# Round 2v: crowd-aware auto mode — GPU tests, then the full default bench (headline + sweep).
out=gpurun_out/r2v; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step pytest 500 python -u -m pytest tests/test_gpu_limits.py tests/test_gpu_e2e.py -k "auto_mode or live_cu or slice or launch_block" -v -s --timeout 200 --timeout-method thread
step bench 600 python -u bench.py
