#!/bin/bash
# Round 2m: launch-bound suite cases after the launch fast path, workers pinned to the
# GPU's NUMA-local CPUs (7 ABBA repeats); then the default bench.py.
out=gpurun_out/r2m; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step suite_lb 700 python -u benchmarks/aibench_suite.py --cases resnet152-inf,resnet152-train,deeplab-train --modes native,vgpu --repeats 7 --vdm 0 --json-out $out/suite_lb.json --md-out $out/suite_lb.md
step bench 480 python -u bench.py
