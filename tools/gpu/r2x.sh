#!/bin/bash
# Round 2x: full default bench under the crowd-aware auto mode.
out=gpurun_out/r2x; mkdir -p $out
timeout -k 10 1000 python -u bench.py > $out/bench.log 2>&1
echo "bench rc=$?" >> $out/steps.txt
