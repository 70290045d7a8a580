#!/bin/bash
# Round 2ac: split-4 pods arriving one by one (1..4): the auto mode's CU masks while the
# GPU is not crowded, the GPU-time limiter from 3 busy pods on.
out=gpurun_out/r2ac; mkdir -p $out
timeout -k 10 800 python -u benchmarks/vgpu_scaling.py --policy default --split 4 --tenants 1,2,3,4 --json-out $out/split4.json --md-out $out/split4.md > $out/split4.log 2>&1
echo "split4 rc=$?" >> $out/steps.txt
