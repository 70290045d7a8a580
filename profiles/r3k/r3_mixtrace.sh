#!/bin/bash
# Round-3: where does the latency pod's time go next to the trainers? Kernel traces of the
# inference service (rocprofv3 --kernel-trace --stats): alone in its split-4 vGPU, then in
# the mix (default and with priority classes), summarised on the box (traces are large:
# only the summaries and per-kernel stats come back). Then the new GPU tests.
out=${1:-gpurun_out/r3k}
mkdir -p "$out"
export TMPDIR=/tmp
P="resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2"
T=/tmp/r3k-traces
rm -rf "$T"
timeout -k 10 300 python -u benchmarks/mix.py --pods resnet50-inf:1:lat --split 4 --seconds 8 --ab 1 \
  --priority "$P" --trace-latency "$T/solo" --json-out "$out/solo.json" --md-out "$out/solo.md" > "$out/solo.log" 2>&1 &&
python tools/probe/lat_kernels.py "$T/solo" --steps-json "$out/solo.json" --out "$out/solo_kernels.json" > "$out/solo_kernels.log" 2>&1 &&
timeout -k 10 600 python -u benchmarks/mix.py --seconds 8 --ab 2 --priority "$P" --trace-latency "$T/mix" \
  --json-out "$out/mix.json" --md-out "$out/mix.md" > "$out/mix.log" 2>&1 &&
python tools/probe/lat_kernels.py "$T/mix" --steps-json "$out/mix.json" --out "$out/mix_kernels.json" > "$out/mix_kernels.log" 2>&1 &&
rm -rf "$T" &&
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread -m gpu \
  "tests/test_gpu_limits.py::test_background_class_yields_to_a_busy_latency_class" \
  "tests/test_gpu_limits.py::test_temporal_four_light_tenants" -p no:cacheprovider > "$out/pytest.log" 2>&1
