#!/bin/bash
# --gpu-concurrency=auto with bursty containers kept out of the turns: the latency mix without
# and with classes (ABAB x3), four LSTM pods (pairs must still switch on), and the GPU pair test.
set -o pipefail
TAG=${1:-r6a2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u benchmarks/mix.py --seconds 8 --ab 3 --gpu-concurrency auto \
  --priority "resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2" \
  --json-out $OUT/mix.json --md-out $OUT/mix.md > $OUT/mix.log 2>&1 || { tail -5 $OUT/mix.log; exit 1; }
tail -10 $OUT/mix.md
grep -c "kept out of the pair turns" $OUT/mix.log
timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 10 --warmup 20 --tenants 4 \
  --pod-env VGPU_GPU_CONCURRENCY=auto --pod-env VGPU_LOG_LEVEL=2 --json-out $OUT/lstm4.json --md-out $OUT/lstm4.md > $OUT/lstm4.log 2>&1 \
  && tail -1 $OUT/lstm4.md && grep -c "pair turns" $OUT/lstm4.log || exit 1
grep "kept out" $OUT/lstm4.log | head -3
timeout -k 10 200 python -u -m pytest tests/test_gpu_pairs.py -x -v -s --timeout 180 --timeout-method thread -p no:cacheprovider > $OUT/pairs_test.log 2>&1; rc=$?
tail -5 $OUT/pairs_test.log; exit $rc
