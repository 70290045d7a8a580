#!/bin/bash
# Pair turns (--gpu-concurrency=2, cross-socket since round 6) vs all-at-once, default policy:
# GPU-bound ResNet-50 b=50 pods at 4 / 8 / 16 per GPU, and launch-bound LSTM pods at 4 / 8 again.
set -o pipefail
TAG=${1:-r6k2}
OUT=gpurun_out/$TAG; mkdir -p $OUT
S="timeout -k 10 500 python -u benchmarks/vgpu_scaling.py --policy default --seconds 6"
$S --case resnet50-inf --tenants 4,8,16 --json-out $OUT/r50_all.json --md-out $OUT/r50_all.md > $OUT/r50_all.log 2>&1 && tail -4 $OUT/r50_all.md &&
$S --case resnet50-inf --tenants 4,8,16 --pod-env VGPU_GPU_CONCURRENCY=2 --json-out $OUT/r50_conc2.json --md-out $OUT/r50_conc2.md > $OUT/r50_conc2.log 2>&1 && tail -4 $OUT/r50_conc2.md &&
$S --case lstm-inf --tenants 1,4,8 --pod-env VGPU_GPU_CONCURRENCY=2 --json-out $OUT/lstm_conc2.json --md-out $OUT/lstm_conc2.md > $OUT/lstm_conc2.log 2>&1 && tail -4 $OUT/lstm_conc2.md
