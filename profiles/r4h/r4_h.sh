#!/bin/bash
# Round-4 GPU study (profiles/r4h): why two concurrent 50 % pods of launch-bound cases run at
# half speed each (r4d VDM column; round 2 ran them nearly in parallel). Pairs of stock
# LSTM / DeepLab inference pods of a split-2 plugin: default policy (each on its disjoint
# 128-CU mask) vs quota-only pods (no mask, no limiter), and each case alone.
out=${1:-gpurun_out/r4h}
mkdir -p "$out"
for c in lstm-inf deeplab-inf; do
  timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case $c --tenants 1,2 --policy default,shared \
    --seconds 6 --json-out "$out/pair_$c.json" --md-out "$out/pair_$c.md" > "$out/pair_$c.log" 2>&1 || exit $?
done
