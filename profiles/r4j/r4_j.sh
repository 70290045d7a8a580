#!/bin/bash
# Round-4 GPU study (profiles/r4j): fairness of 16 crowded pods (thin shares: time-sliced on
# every CU, full CU count - the round-4 default) with at most K containers' GPU-time gates open
# at once (VGPU_GPU_CONCURRENCY; the hardware scheduler maps a limited number of processes at
# once, hws.txt), K = unbounded / 8 / 4.
out=${1:-gpurun_out/r4j}
what=${2:-conc0,conc8,conc4}
mkdir -p "$out"
for k in 0 8 4; do
  [[ $what == *conc$k* ]] || continue
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_GPU_CONCURRENCY=$k --json-out "$out/conc${k}_16.json" --md-out "$out/conc${k}_16.md" \
    > "$out/conc${k}_16.log" 2>&1 || exit $?
done
