#!/bin/bash
# Round 2ad: 3 busy split-4 pods under CU masks vs the limiter (auto's crowd threshold).
out=gpurun_out/r2ad; mkdir -p $out
timeout -k 10 600 python -u benchmarks/vgpu_scaling.py --policy spatial --split 4 --tenants 3 --repeats 2 --json-out $out/spatial3.json --md-out $out/spatial3.md > $out/spatial3.log 2>&1
echo "spatial3 rc=$?" >> $out/steps.txt
