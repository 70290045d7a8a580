#!/bin/bash
# Round 2j: spill + smi tests, hook overhead after the launch fast path, rocprofv3 tenant
# profiles (resnet50-inf modes; resnet152-train process-to-process variation).
out=gpurun_out/r2j; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 400 python -u -m pytest "tests/test_gpu_limits.py::test_spill_placement_policy" "tests/test_gpu_e2e.py::test_amdsmi_shows_only_the_containers_gpus_and_processes" "tests/test_gpu_limits.py::test_launch_counter_and_hostpids_for_simultaneous_starters" -v -s --timeout 200 --timeout-method thread
step hooks 400 python -u benchmarks/hook_overhead.py --json-out $out/hooks.json --md-out $out/hooks.md
step prof 500 python -u tools/probe/prof_tenant.py --out $out/prof
step prof152 600 python -u tools/probe/prof_tenant.py --out $out/prof152 --case resnet152-train --modes native,vgpu-quota --runs 3 --steps 20
