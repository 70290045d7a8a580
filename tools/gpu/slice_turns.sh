#!/bin/bash
# Turn length of the pair turns (VGPU_GPU_SLICE_MS, default 20) for 4 and 8 LSTM pods under
# --gpu-concurrency=auto, ABAB: 20 ms vs 40 ms (SLICES="20 10" for others).
set -o pipefail
TAG=${1:-r6x}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for n in 4 8; do
  for r in 1 2; do
    for s in ${SLICES:-20 40}; do
      timeout -k 10 240 python -u benchmarks/vgpu_scaling.py --case lstm-inf --policy default --seconds 10 --warmup 20 --tenants $n \
        --pod-env VGPU_GPU_CONCURRENCY=auto --pod-env VGPU_GPU_SLICE_MS=$s --pod-env VGPU_STATS=1 \
        --json-out $OUT/lstm${n}_s${s}_$r.json --md-out $OUT/lstm${n}_s${s}_$r.md > $OUT/lstm${n}_s${s}_$r.log 2>&1 || exit 1
      echo "n=$n slice=$s run=$r: $(tail -1 $OUT/lstm${n}_s${s}_$r.md | cut -c1-160)"
    done
  done
done
