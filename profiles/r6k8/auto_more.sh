#!/bin/bash
# After the board clock fix, with auto as the default: eight LSTM pods (auto vs off), and four
# tiny-kernel pods (auto, default wait).
set -o pipefail
TAG=${1:-r6k8}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
S="timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 10 --warmup 20"
$S --tenants 1,8 --gpu-concurrency auto --json-out $OUT/lstm8_auto.json --md-out $OUT/lstm8_auto.md > $OUT/lstm8_auto.log 2>&1 && tail -2 $OUT/lstm8_auto.md | cut -c1-200 || exit 1
$S --tenants 8 --gpu-concurrency 0 --json-out $OUT/lstm8_off.json --md-out $OUT/lstm8_off.md > $OUT/lstm8_off.log 2>&1 && tail -1 $OUT/lstm8_off.md | cut -c1-200 || exit 1
timeout -k 10 120 python3 benchmarks/tiny_pods.py --pods 4 --conc auto --seconds 4 > $OUT/tiny_auto.json 2> $OUT/tiny.err || exit 1
python3 -c "import json; d=json.load(open('$OUT/tiny_auto.json')); print('tiny auto', d['aggregate_kps'], [p['kps'] for p in d['per_pod']])"
