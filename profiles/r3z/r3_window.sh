#!/bin/bash
# Round-3: 12 crowded pods, the limiter's credit window 40 ms (shipped) vs 150 ms, with the
# crowd-stretched sampling period of the shipped shim (r2ae measured 150 ms only at a fixed
# 1 ms period). Two repeats, ABAB order within each.
out=${1:-gpurun_out/r3z}
reps=${2:-2}
mkdir -p "$out"
timeout -k 10 1080 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants 1,12 \
  --repeats "$reps" --pod-env "VGPU_LIMITER_WINDOW_MS=40,150" --json-out "$out/window.json" \
  --md-out "$out/window.md" > "$out/window.log" 2>&1
