#!/bin/bash
# Round 2aa: the ten-case suite in one run on the final round-2 shim (5 ABBA repeats + VDM).
out=gpurun_out/r2aa; mkdir -p $out
timeout -k 10 1150 python -u benchmarks/aibench_suite.py --cases all --repeats 5 --json-out $out/suite.json --md-out $out/suite.md > $out/suite.log 2>&1
echo "suite rc=$?" >> $out/steps.txt
