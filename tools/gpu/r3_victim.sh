#!/bin/bash
# Round-3: does the board's CU reservation keep a background pod's work off the latency
# pod's slice on real hardware, and does that protect the latency pod's kernels?
#   1. GPU tests: the reservation census, then the background-yield test.
#   2. The b=1 service next to one VGG-16 trainer with no compute share (whole GPU):
#      default (trainer on all 256 CUs) vs priority (service 0 on its 64-CU slice, trainer
#      2 = background: re-masked to the other 192 CUs; with no share it is not time-gated),
#      kernel traces of the service summarised on the box.
out=${1:-gpurun_out/r3l}
mkdir -p "$out"
export TMPDIR=/tmp
T=/tmp/r3l-traces
rm -rf "$T"
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread -m gpu \
  "tests/test_gpu_limits.py::test_background_class_keeps_off_the_latency_slice" -p no:cacheprovider \
  > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 500 python -u benchmarks/mix.py --pods resnet50-inf:1:lat vgg16-train:nolimit --split 4 --seconds 8 \
  --ab 2 --priority "resnet50-inf:1:lat=0,vgg16-train:nolimit=2" --trace-latency "$T/v" \
  --json-out "$out/victim.json" --md-out "$out/victim.md" > "$out/victim.log" 2>&1 &&
python tools/probe/lat_kernels.py "$T/v" --steps-json "$out/victim.json" --out "$out/victim_kernels.json" \
  > "$out/victim_kernels.log" 2>&1
rm -rf "$T"
