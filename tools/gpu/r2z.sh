#!/bin/bash
# Round 2z: 8 crowded pods, CU count virtualised (slice) vs real, 2 repeats each.
out=gpurun_out/r2z; mkdir -p $out
timeout -k 10 1000 python -u benchmarks/vgpu_scaling.py --policy default --tenants 1,8 --pod-env VGPU_VIRTUAL_CU_COUNT=1,0 --repeats 2 --json-out $out/virt.json --md-out $out/virt.md > $out/virt.log 2>&1
echo "virt rc=$?" >> $out/steps.txt
