#!/bin/bash
# Round-3 many-pod repeats (profiles/r3g): the shipped limiter vs the board's concurrency
# admission (k = 2) at 8, 12 and 16 crowded ResNet-50 pods, two repeats.
out=${1:-gpurun_out/r3g}
mkdir -p "$out"
run() {
  local tag=$1
  shift
  timeout -k 10 560 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --json-out "$out/$tag.json" \
    --md-out "$out/$tag.md" "$@" > "$out/$tag.log" 2>&1
}
run k0 --tenants 1,12,16 --repeats 2 && run k2 --tenants 8,12,16 --repeats 2 --pod-env VGPU_GPU_CONCURRENCY=2
