#!/bin/bash
# Round 2n: concurrent-pod scaling curve per --cu-mode policy (stock fp32 ResNet-50
# inference), then bench.py with the rounded-up CU shares.
out=gpurun_out/r2n; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step scaling 800 python -u benchmarks/vgpu_scaling.py --policy default,spatial,shared --json-out $out/scaling.json --md-out $out/scaling.md
step bench 400 python -u bench.py
