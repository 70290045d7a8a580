#!/bin/bash
# Round 2f: round-2 GPU tests (stock 2-tenant accuracy, IPC), limiter window comparison.
out=gpurun_out/r2f; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 700 python -u -m pytest tests/test_gpu_limits.py -v -s --timeout 300 --timeout-method thread
step w120 400 python -u benchmarks/temporal_accuracy.py --workload resnet50 --limits 10,25,50 --tenants 1 --extra VGPU_LIMITER_WINDOW_MS=120 --json-out $out/temporal_w120.json --md-out $out/temporal_w120.md
step w40 400 python -u benchmarks/temporal_accuracy.py --workload resnet50 --limits 10,25,50 --tenants 1 --json-out $out/temporal_w40.json --md-out $out/temporal_w40.md
