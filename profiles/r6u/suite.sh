#!/bin/bash
# The ten-case suite at HEAD (as profiles/r4d): native / vgpu (interception only) / vgpu-cu50
# (the reference DaemonSet's contract) in ABBA order with 95 % CIs, plus the two-pod VDM
# column; every contract from a real Allocate.
set -o pipefail
TAG=${1:-r6u}; REPS=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 1140 python -u benchmarks/aibench_suite.py --cases all --repeats "$REPS" --json-out "$OUT/suite.json" \
  --md-out "$OUT/suite.md" > "$OUT/suite.log" 2>&1
rc=$?; tail -16 $OUT/suite.log; exit $rc
