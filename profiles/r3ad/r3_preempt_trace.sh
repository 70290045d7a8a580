#!/bin/bash
# Round-3: kernel traces of the inference service in the mix under the shipped strict
# preemption of the background class (hold 3 ms, depth 4) against the soft yield
# (VGPU_PREEMPT_HOLD_MS=0, VGPU_PREEMPT_DEPTH=0): does the service's own kernel time per
# request come back toward its solo 1.7 ms (r3k: 4.6-5.4 ms next to the trainers)?
# rocprofv3 --kernel-trace --stats of the latency pod only; summaries come back.
out=${1:-gpurun_out/r3ad}
mkdir -p "$out"
export TMPDIR=/tmp
P="resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2"
T=/tmp/r3ad-traces
rm -rf "$T"
timeout -k 10 700 python -u benchmarks/mix.py --seconds 8 --ab 2 --skip-default --priority "$P" \
  --bg-env VGPU_PREEMPT_HOLD_MS=0,VGPU_PREEMPT_DEPTH=0 --trace-latency "$T/mix" \
  --json-out "$out/mix.json" --md-out "$out/mix.md" > "$out/mix.log" 2>&1 &&
python tools/probe/lat_kernels.py "$T/mix" --steps-json "$out/mix.json" --out "$out/mix_kernels.json" > "$out/mix_kernels.log" 2>&1
rc=$?
rm -rf "$T"
exit $rc
