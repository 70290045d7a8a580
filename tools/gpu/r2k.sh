#!/bin/bash
# Round 2k: spill placement after the double-count fix; rocprofv3 tenant profiles
# (resnet50-inf modes; resnet152-train process-to-process variation, autotune on / off).
out=gpurun_out/r2k; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 300 python -u -m pytest "tests/test_gpu_limits.py::test_spill_placement_policy" -v -s --timeout 200 --timeout-method thread
step prof 500 python -u tools/probe/prof_tenant.py --out $out/prof
step prof152 600 python -u tools/probe/prof_tenant.py --out $out/prof152 --case resnet152-train --modes native,vgpu-quota --runs 3 --steps 20
step prof152h 600 python -u tools/probe/prof_tenant.py --out $out/prof152h --case resnet152-train --modes native,vgpu-quota --runs 3 --steps 20 --autotune 0
