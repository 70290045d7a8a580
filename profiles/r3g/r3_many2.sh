#!/bin/bash
# Round-3 many-pod repeats (profiles/r3g): the shipped limiter (k0) vs the board's
# concurrency admission (k2: two gates open at once) for crowded ResNet-50 pods.
#   bash profiles/r3g/r3_many2.sh <out> <tenants> <repeats>
out=${1:-gpurun_out/r3g}
tenants=${2:-12}
reps=${3:-2}
mkdir -p "$out"
run() {
  local tag=$1
  shift
  timeout -k 10 560 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --json-out "$out/$tag.json" \
    --md-out "$out/$tag.md" "$@" > "$out/$tag.log" 2>&1
}
run "k0_$tenants" --tenants "1,$tenants" --repeats "$reps" &&
  run "k2_$tenants" --tenants "$tenants" --repeats "$reps" --pod-env VGPU_GPU_CONCURRENCY=2
