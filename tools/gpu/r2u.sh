#!/bin/bash
# Round 2u: a lone split-4 pod under a spatial 25 % mask vs the temporal limiter.
out=gpurun_out/r2u; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step spatial 300 python -u bench.py --modes native,vgpu --cu-mode spatial --sweep off --steps 40
step temporal 300 python -u bench.py --modes native,vgpu --cu-mode temporal --sweep off --steps 40
