#!/bin/bash
# Round 2h: spill placement tests + config-4 benchmark with the ResNet policy study.
out=gpurun_out/r2h; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 300 python -u -m pytest tests/test_gpu_limits.py -k spill -v -s --timeout 200 --timeout-method thread
step oversub 1000 python -u benchmarks/oversubscribe.py --json-out $out/oversub.json --md-out $out/oversub.md
