#!/bin/bash
# After the heartbeat fix: the default bench (16-pod sweep on the node ledger), four LSTM pods
# under --gpu-concurrency=auto twice, and the latency mix with auto (ABAB x3).
set -o pipefail
TAG=${1:-r6a5}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
bash tools/gpu/session.sh $TAG bench || exit 1
for r in 1 2; do
  timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 10 --warmup 20 --tenants 4 \
    --pod-env VGPU_GPU_CONCURRENCY=auto --pod-env VGPU_LOG_LEVEL=2 --pod-env VGPU_STATS=1 --json-out $OUT/lstm4_$r.json \
    --md-out $OUT/lstm4_$r.md > $OUT/lstm4_$r.log 2>&1 || exit 1
  tail -1 $OUT/lstm4_$r.md | cut -c1-200; echo "pair on/off msgs: $(grep -c 'pair turns\|all at once' $OUT/lstm4_$r.log) bursty: $(grep -c 'bursty' $OUT/lstm4_$r.log)"
done
timeout -k 10 900 python -u benchmarks/mix.py --seconds 8 --ab 3 --gpu-concurrency auto \
  --priority "resnet50-inf:1:lat=0,vgg16-train=2,lstm-train=2,deeplab-inf=2" \
  --json-out $OUT/mix.json --md-out $OUT/mix.md > $OUT/mix.log 2>&1 || { tail -5 $OUT/mix.log; exit 1; }
tail -10 $OUT/mix.md
