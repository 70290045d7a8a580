#!/bin/bash
# Round-4 GPU study (profiles/r4y): where the 12- and 16-pod throughput spread comes from.
# The bench's sweep setup (ledger default, auto policy, MIOpen immediate mode, per-pod
# find-db), with each pod's GPU time as the limiter charged it (granted %) and its images per
# charged GPU-ms, 2 repeats.
out=${1:-gpurun_out/r4y}
mkdir -p "$out"
VGPU_BENCH_AUTOTUNE=0 timeout -k 10 600 python -u benchmarks/vgpu_scaling.py --policy default --tenants 1,12,16 \
  --repeats 2 --miopen-db per-pod --json-out "$out/spread.json" --md-out "$out/spread.md" > "$out/spread.log" 2>&1
echo "spread_rc=$?" >> "$out/spread.log"
