#!/bin/bash
# Round 2i: fixed spill / amd-smi tests, then the 10-case suite (first half) with ABBA repeats + VDM.
out=gpurun_out/r2i; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
}
step pytest 300 python -u -m pytest tests/test_gpu_limits.py -k spill tests/test_gpu_e2e.py::test_amdsmi_shows_only_the_containers_gpus_and_processes -v -s --timeout 200 --timeout-method thread
step suite_a 1000 python -u benchmarks/aibench_suite.py --cases resnet50-inf,resnet50-train,resnet152-inf,resnet152-train,vgg16-inf --repeats 5 --json-out $out/suite_a.json --md-out $out/suite_a.md
