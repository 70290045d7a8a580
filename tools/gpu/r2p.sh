#!/bin/bash
# Round 2p: limiter window sweep (per-cycle warm-up cost vs window) for the bench tenant.
out=gpurun_out/r2p; mkdir -p $out
timeout -k 10 700 python -u tools/probe/limiter_trace.py --limits 99,25,10 --windows 40,100,200 --steps 60 --out $out/windows.json > $out/windows.log 2>&1
echo "windows rc=$?" >> $out/steps.txt
