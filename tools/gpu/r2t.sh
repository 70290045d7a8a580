#!/bin/bash
# Round 2t (2): 8 spatial pods with the virtual CU count; parity pod.
out=gpurun_out/r2t; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step spatial8 600 python -u benchmarks/vgpu_scaling.py --policy spatial --tenants 8 --json-out $out/spatial8.json --md-out $out/spatial8.md
step bench 300 python -u bench.py --modes native,parity --sweep off
