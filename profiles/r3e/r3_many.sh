#!/bin/bash
# Round-3 many-pod study (profiles/r3e): 12 crowded split-12 ResNet-50 pods under the
# default auto policy (GPU-time limiter): the shipped limiter, a longer limiter window,
# the progress charge, and the board's concurrency admission (k gates open at once).
out=${1:-gpurun_out/r3e}
what=${2:-base,window,progress,conc}
mkdir -p "$out"
run() {
  local tag=$1
  shift
  timeout -k 10 500 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --json-out "$out/$tag.json" \
    --md-out "$out/$tag.md" "$@" > "$out/$tag.log" 2>&1
}
set -e
[[ $what == *base* ]] && run base --tenants 1,12
[[ $what == *conc* ]] && run conc --tenants 12 --pod-env VGPU_GPU_CONCURRENCY=2,4
[[ $what == *window* ]] && run window --tenants 12 --pod-env VGPU_LIMITER_WINDOW_MS=150
[[ $what == *progress* ]] && run progress --tenants 12 --pod-env VGPU_CHARGE_MODEL=progress
exit 0
