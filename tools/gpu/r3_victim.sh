#!/bin/bash
# Round-3: does the board's CU reservation keep a background pod's work off the latency
# pod's slice on real hardware, and does that protect the latency pod's kernels?
#   1. GPU test: the reservation census.
#   2. The b=1 service next to one VGG-16 trainer with no compute share (whole GPU):
#      default (trainer on all 256 CUs) vs priority (service 0 on its 64-CU slice, trainer
#      2 = background: re-masked to the other 192 CUs; with no share it is not time-gated),
#      the service's per-request GPU time from HIP events (no profiler).
out=${1:-gpurun_out/r3l}
mkdir -p "$out"
export TMPDIR=/tmp


timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread -m gpu \
  "tests/test_gpu_limits.py::test_background_class_keeps_off_the_latency_slice" -p no:cacheprovider \
  > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 500 python -u benchmarks/mix.py --pods resnet50-inf:1:lat vgg16-train:nolimit --split 4 --seconds 8 \
  --ab 3 --priority "resnet50-inf:1:lat=0,vgg16-train:nolimit=2" \
  --json-out "$out/victim.json" --md-out "$out/victim.md" > "$out/victim.log" 2>&1
rc=$?
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u benchmarks/mix.py --pods resnet50-inf:1:lat --split 4 --seconds 8 --ab 1 \
  --priority "resnet50-inf:1:lat=0" --json-out "$out/solo.json" --md-out "$out/solo.md" > "$out/solo.log" 2>&1
