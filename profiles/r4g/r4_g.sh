#!/bin/bash
# Round-4 GPU study (profiles/r4g): where 16 crowded pods' ~200 s start-up goes. Every pod is
# told the GPU's full CU count (VGPU_VIRTUAL_CU_COUNT=0, r4c: 1.01x aggregate, slowest 0.92).
#   nolimit  16 pods with quotas only (no CU mask, no GPU-time limiter): start-up without the
#            limiter, on an empty find-db (fills ~/.config/miopen for the full CU count)
#   perpod   16 pods on the default policy, each with its own copy of that find-db and kernel
#            cache (a tenant image with a tuned find-db; no sqlite shared between pods)
#   conc8    16 pods, default policy, at most 8 containers' GPU-time gates open at once
out=${1:-gpurun_out/r4g}
what=${2:-nolimit,perpod}
mkdir -p "$out"
if [[ $what == *nolimit* ]]; then
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy shared --tenants 16 --seconds 8 \
    --pod-env VGPU_VIRTUAL_CU_COUNT=0 --json-out "$out/nolimit_16.json" --md-out "$out/nolimit_16.md" \
    > "$out/nolimit_16.log" 2>&1 || exit $?
fi
if [[ $what == *perpod* ]]; then
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_VIRTUAL_CU_COUNT=0 --miopen-db per-pod --json-out "$out/perpod_16.json" \
    --md-out "$out/perpod_16.md" > "$out/perpod_16.log" 2>&1 || exit $?
fi
if [[ $what == *conc8* ]]; then
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_VIRTUAL_CU_COUNT=0 --pod-env VGPU_GPU_CONCURRENCY=8 --json-out "$out/conc8_16.json" \
    --md-out "$out/conc8_16.md" > "$out/conc8_16.log" 2>&1 || exit $?
fi
