#!/bin/bash
# Round 2s: does HW-queue oversubscription explain the collapse of many pods? KFD queue
# counts and GPU_MAX_HW_QUEUES 1 vs default at 8 (shared) and 12 (default) pods.
out=gpurun_out/r2s; mkdir -p $out
timeout -k 10 1000 python -u benchmarks/vgpu_scaling.py --policy shared,default --tenants 1,8,12 --hw-queues 0,1 --json-out $out/hwq.json --md-out $out/hwq.md > $out/hwq.log 2>&1
echo "hwq rc=$?" >> $out/steps.txt
