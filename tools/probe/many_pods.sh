#!/bin/bash
# Many-pod limiter study (profiles/r2ad): 12 crowded split-12 pods under the default auto
# policy, varying the occupancy sampling period and the limiter window, to find where
# the 12-pod aggregate (0.88x in profiles/r2s) loses throughput.
# Usage (GPU box): bash tools/probe/many_pods.sh <outdir>
set -o pipefail
out=${1:-gpurun_out/many_pods}
mkdir -p "$out"
run() {
  local tag=$1
  shift
  timeout -k 10 420 python -u benchmarks/vgpu_scaling.py --policy default --json-out "$out/$tag.json" \
    --md-out "$out/$tag.md" "$@" > "$out/$tag.log" 2>&1
}
run base --tenants 1,12 &&
  run sample4ms --tenants 12 --pod-env VGPU_UTIL_SAMPLE_US=4000 &&
  run window150 --tenants 12 --pod-env VGPU_LIMITER_WINDOW_MS=150
