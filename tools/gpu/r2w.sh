#!/bin/bash
# Round 2w: 8-pod sweep point under the crowd-aware auto mode (warm-up time, modes).
out=gpurun_out/r2w; mkdir -p $out
timeout -k 10 900 python -u bench.py --modes native --sweep on --sweep-tenants 1,8 > $out/bench8.log 2>&1
echo "bench8 rc=$?" >> $out/steps.txt
