#!/bin/bash
# One noisy suite case re-measured (as profiles/r5f): native vs the quota-only vGPU, 8 ABBA
# repeats of a 10 s timed window each; then bench.py --gpus 2 on this one-GPU box must refuse.
set -o pipefail
TAG=${1:-r6u2}; C=${2:-resnet152-train}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1000 python -u benchmarks/aibench_suite.py --cases $C --modes native,vgpu --repeats 8 --window 10 \
  --vdm 0 --json-out $OUT/$C.json --md-out $OUT/$C.md > $OUT/$C.log 2>&1 || { tail -5 $OUT/$C.log; exit 1; }
tail -6 $OUT/$C.log
timeout -k 10 120 python bench.py --gpus 2 > $OUT/gpus2.log 2>&1; echo "bench --gpus 2 rc=$?" | tee -a $OUT/gpus2.log; tail -2 $OUT/gpus2.log
