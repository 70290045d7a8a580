#!/bin/bash
# --gpu-concurrency=auto on 4 LSTM pods, 10 s windows after 20 warm-up steps, three repeats,
# against all at once (ABAB...): is the pair-turn gain steady?
set -o pipefail
TAG=${1:-r6k7}
OUT=gpurun_out/$TAG; mkdir -p $OUT
S="timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 10 --warmup 20 --tenants 4"
pt() { tail -1 $OUT/$1.md | awk -F'|' '{print "'$1'", $8, $9, $11}'; }
for r in 1 2 3; do
  $S --pod-env VGPU_GPU_CONCURRENCY=auto --json-out $OUT/auto_$r.json --md-out $OUT/auto_$r.md > $OUT/auto_$r.log 2>&1 && pt auto_$r || exit 1
  $S --json-out $OUT/all_$r.json --md-out $OUT/all_$r.md > $OUT/all_$r.log 2>&1 && pt all_$r || exit 1
done
