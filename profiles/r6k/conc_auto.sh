#!/bin/bash
# --gpu-concurrency=auto (VGPU_GPU_CONCURRENCY=auto): pair turns only while a GPU's pods launch
# more than 40k kernels/s together. Launch-bound LSTM pods (4 twice, 8) and GPU-bound ResNet-50
# b=50 pods (4, 8, 16); info logs show when pairs switch on.
set -o pipefail
TAG=${1:-r6k6}
OUT=gpurun_out/$TAG; mkdir -p $OUT
S="timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --policy default --seconds 6 --pod-env VGPU_GPU_CONCURRENCY=auto --pod-env VGPU_LOG_LEVEL=2"
pt() { tail -$2 $OUT/$1.md | awk -F'|' '{print "'$1'", $8, $9, $11}'; echo "pairs on: $(grep -c 'pair turns' $OUT/$1.log), off: $(grep -c 'all at once' $OUT/$1.log)"; }
$S --case lstm-inf --tenants 4 --json-out $OUT/lstm4a.json --md-out $OUT/lstm4a.md > $OUT/lstm4a.log 2>&1 && pt lstm4a 1 || exit 1
$S --case lstm-inf --tenants 4,8 --json-out $OUT/lstm48.json --md-out $OUT/lstm48.md > $OUT/lstm48.log 2>&1 && pt lstm48 2 || exit 1
$S --case resnet50-inf --tenants 4,8,16 --json-out $OUT/r50.json --md-out $OUT/r50.md > $OUT/r50.log 2>&1 && pt r50 3 || exit 1
