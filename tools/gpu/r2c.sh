#!/bin/bash
# Round 2c: sampler overhead + temporal accuracy with gate hysteresis (+ spin workload).
out=gpurun_out/r2c; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step overhead 300 python -u tools/probe/sampler_overhead.py --out $out/sampler_overhead.json
step temporal 600 python -u benchmarks/temporal_accuracy.py --workload resnet50 --limits 10,25,50,75,90 --tenants 1,2 --json-out $out/temporal.json --md-out $out/temporal.md
step temporal_spin 300 python -u benchmarks/temporal_accuracy.py --workload spin --limits 10,25,50,75 --tenants 1 --json-out $out/temporal_spin.json --md-out $out/temporal_spin.md
