#!/bin/bash
# Pair turns vs all at once on LSTM pods, alternating (ABAB) at 4 pods, then 8 pods each way.
set -o pipefail
TAG=${1:-r6k5}
OUT=gpurun_out/$TAG; mkdir -p $OUT
S="timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 6"
pt() { tail -1 $OUT/$1.md | awk -F'|' '{print "'$1'", $8, $9, $11}'; }
for r in 1 2; do
  $S --tenants 4 --pod-env VGPU_GPU_CONCURRENCY=2 --json-out $OUT/conc4_$r.json --md-out $OUT/conc4_$r.md > $OUT/conc4_$r.log 2>&1 && pt conc4_$r || exit 1
  $S --tenants 4 --json-out $OUT/all4_$r.json --md-out $OUT/all4_$r.md > $OUT/all4_$r.log 2>&1 && pt all4_$r || exit 1
done
$S --tenants 8 --pod-env VGPU_GPU_CONCURRENCY=2 --json-out $OUT/conc8.json --md-out $OUT/conc8.md > $OUT/conc8.log 2>&1 && pt conc8 || exit 1
$S --tenants 1,8 --json-out $OUT/all8.json --md-out $OUT/all8.md > $OUT/all8.log 2>&1 && tail -2 $OUT/all8.md
