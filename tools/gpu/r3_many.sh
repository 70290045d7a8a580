#!/bin/bash
# Round-3 many-pod study (profiles/r3e): 12 crowded split-12 ResNet-50 pods under the
# default auto policy (GPU-time limiter), varying the limiter window and charge model.
out=${1:-gpurun_out/r3e}
mkdir -p "$out"
run() {
  local tag=$1
  shift
  timeout -k 10 500 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --json-out "$out/$tag.json" \
    --md-out "$out/$tag.md" "$@" > "$out/$tag.log" 2>&1
}
run base --tenants 1,12 &&
  run window --tenants 12 --pod-env VGPU_LIMITER_WINDOW_MS=150,400 &&
  run progress --tenants 12 --pod-env VGPU_CHARGE_MODEL=progress
