#!/bin/bash
# Round 2b: shim/control/e2e GPU tests after the limiter redesign + temporal accuracy.
out=gpurun_out/r2b; mkdir -p $out
step() {  # step <name> <timeout> <cmd...>: run; stop the script on anything but pass/test-failure
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" | tee -a $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 900 python -u -m pytest tests/test_gpu_shim.py tests/test_gpu_control.py tests/test_gpu_e2e.py -x -v --timeout 120 --timeout-method thread
step temporal 600 python -u benchmarks/temporal_accuracy.py --workload resnet50 --json-out $out/temporal.json --md-out $out/temporal.md
