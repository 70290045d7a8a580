#!/bin/bash
# Round-3: 16 crowded pods of a split-16 plugin. Does the rounded-up share (7 % each,
# 112 % in total) let some pods take more than 1/16 of the GPU's time? Same pods with the
# share overridden to 6 % (96 % in total); per-pod granted GPU time is in the JSON.
#   bash profiles/r3n/r3_sixteen.sh <out> [shares]
out=${1:-gpurun_out/r3n}
shares=${2:-7,6}
mkdir -p "$out"
timeout -k 10 900 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants 1,16 \
  --pod-env "VGPU_DEVICE_CU_LIMIT_0=$shares" --json-out "$out/sixteen.json" --md-out "$out/sixteen.md" \
  > "$out/sixteen.log" 2>&1
