#!/bin/bash
# Round-4 ten-case suite at HEAD (profiles/r4d): native / vgpu (interception only) /
# vgpu-cu50 (the reference DaemonSet's contract) in ABBA order with 95 % CIs, plus the
# two-pod VDM column; the contracts come from real Allocate responses (plugin-owned limits
# file included).
out=${1:-gpurun_out/r4d}
reps=${2:-4}
mkdir -p "$out"
timeout -k 10 1140 python -u benchmarks/aibench_suite.py --cases all --repeats "$reps" --json-out "$out/suite.json" \
  --md-out "$out/suite.md" > "$out/suite.log" 2>&1
echo "suite_rc=$?" >> "$out/suite.log"
