#!/bin/bash
# The GPU pair test, then four LSTM pods under --gpu-concurrency=auto three times with the
# shim's admission statistics (VGPU_STATS: turns, time held / waited, longest wait) per pod.
set -o pipefail
TAG=${1:-r6a3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 200 python -u -m pytest tests/test_gpu_pairs.py -x -v -s --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pairs_test.log 2>&1
rc=$?; grep -E "kps|turns=|passed|failed" $OUT/pairs_test.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
for r in 1 2 3; do
  timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 10 --warmup 20 --tenants 4 \
    --pod-env VGPU_GPU_CONCURRENCY=auto --pod-env VGPU_STATS=1 --json-out $OUT/lstm4_$r.json --md-out $OUT/lstm4_$r.md > $OUT/lstm4_$r.log 2>&1 || exit 1
  tail -1 $OUT/lstm4_$r.md | cut -c1-200; grep -o "turns=.*max_wait_ms=[0-9.]*" $OUT/lstm4_$r.log
done
