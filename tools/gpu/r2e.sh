#!/bin/bash
# Round 2e: re-run the round-2 GPU tests, then the new default bench.py.
out=gpurun_out/r2e; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 600 python -u -m pytest tests/test_gpu_limits.py -v -s --timeout 240 --timeout-method thread
step bench 900 python -u bench.py --json-out $out/bench.json
