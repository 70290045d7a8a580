#!/bin/bash
# Pair turns with the shim's admission decisions logged (VGPU_LOG_LEVEL=3): 4 LSTM pods, twice.
set -o pipefail
TAG=${1:-r6k3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
for r in 1 2; do
  timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --tenants 4 --policy default --seconds 5 \
    --pod-env VGPU_GPU_CONCURRENCY=2 --pod-env VGPU_LOG_LEVEL=3 --json-out $OUT/run$r.json --md-out $OUT/run$r.md \
    > $OUT/run$r.log 2>&1 || { echo "run $r failed"; tail -5 $OUT/run$r.log; exit 1; }
  tail -1 $OUT/run$r.md
  grep -c "admitted after" $OUT/run$r.log
done
