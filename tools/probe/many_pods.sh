#!/bin/bash
# Many-pod limiter study on one MI355X (profiles/r2ae, r2af, r2aj, r2ak).
#
#   bash tools/probe/many_pods.sh <outdir> [study]
#
# study "period" (r2ae): 12 crowded split-12 pods under the default auto policy with the
#   round-2 sampler, a 4 ms sampling period, and a 150 ms limiter window.
# study "efficiency" (default, the next experiment from profiles/r2ak): 8 and 12 pods,
#   12 s windows, two repeats. vgpu_scaling records each pod's granted GPU share and its
#   throughput per charged GPU-millisecond (per_tenant_granted_pct,
#   per_tenant_images_per_gpu_ms), so the 12-pod spread can be split into
#   "got less GPU time" versus "did less per GPU-millisecond".
set -o pipefail
out=${1:-gpurun_out/many_pods}
study=${2:-efficiency}
mkdir -p "$out"
run() {
  local tag=$1
  shift
  timeout -k 10 540 python -u benchmarks/vgpu_scaling.py --policy default --json-out "$out/$tag.json" \
    --md-out "$out/$tag.md" "$@" > "$out/$tag.log" 2>&1
}
if [ "$study" = period ]; then
  run base --tenants 1,12 &&
    run sample4ms --tenants 12 --pod-env VGPU_UTIL_SAMPLE_US=4000 &&
    run window150 --tenants 12 --pod-env VGPU_LIMITER_WINDOW_MS=150
else
  run efficiency --tenants 1,8,12 --seconds 12 --repeats 2
fi
