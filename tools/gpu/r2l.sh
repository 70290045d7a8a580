#!/bin/bash
# Round 2l: ten-case suite, second half (native / vgpu / vgpu-cu50, 5 ABBA repeats, VDM column).
out=gpurun_out/r2l; mkdir -p $out
timeout -k 10 1100 python -u benchmarks/aibench_suite.py --cases deeplab-inf,deeplab-train,lstm-inf,lstm-train,vgg16-train \
  --repeats 5 --json-out $out/suite_b.json --md-out $out/suite_b.md > $out/suite_b.log 2>&1
echo "suite_b rc=$?" >> $out/steps.txt
