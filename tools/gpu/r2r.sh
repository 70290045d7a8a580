#!/bin/bash
# Round 2r: bench after the gloo control group change; 12 concurrent pods; training tenants.
out=gpurun_out/r2r; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step bench 300 python -u bench.py --sweep off
step scal12 400 python -u benchmarks/vgpu_scaling.py --policy default --tenants 1,12 --json-out $out/scal12.json --md-out $out/scal12.md
step scaltrain 500 python -u benchmarks/vgpu_scaling.py --case resnet50-train --policy default,shared --tenants 1,2,4,8 --json-out $out/scaltrain.json --md-out $out/scaltrain.md
