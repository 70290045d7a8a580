#!/bin/bash
# Pair turns (--gpu-concurrency=2, cross-socket) on LSTM pods, the shim's admission decisions
# logged (VGPU_LOG_LEVEL=3): 4 pods twice, 8 pods once; then 4 pods all at once for reference.
set -o pipefail
TAG=${1:-r6k4}
OUT=gpurun_out/$TAG; mkdir -p $OUT
S="timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 5"
for r in 1 2; do
  $S --tenants 4 --pod-env VGPU_GPU_CONCURRENCY=2 --pod-env VGPU_LOG_LEVEL=3 --json-out $OUT/conc4_$r.json \
    --md-out $OUT/conc4_$r.md > $OUT/conc4_$r.log 2>&1 || { echo "run $r failed"; tail -5 $OUT/conc4_$r.log; exit 1; }
  tail -1 $OUT/conc4_$r.md; echo "admissions: $(grep -c 'admitted after' $OUT/conc4_$r.log)"
  gzip -f $OUT/conc4_$r.log
done
$S --tenants 1,8 --pod-env VGPU_GPU_CONCURRENCY=2 --json-out $OUT/conc8.json --md-out $OUT/conc8.md > $OUT/conc8.log 2>&1 \
  && tail -2 $OUT/conc8.md || exit 1
$S --tenants 4 --json-out $OUT/all4.json --md-out $OUT/all4.md > $OUT/all4.log 2>&1 && tail -1 $OUT/all4.md
