#!/bin/bash
# Round-3: the node ledger (one occupancy sampler per node, vgpu-ledger) against every
# container sampling by itself (VGPU_LEDGER=0 in the pods), 12 and 16 crowded pods.
#   bash profiles/r3u/r3_ledger.sh <out> [tenants] [repeats]
out=${1:-gpurun_out/r3u}
tenants=${2:-1,12,16}
reps=${3:-1}
mkdir -p "$out"
timeout -k 10 1080 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants "$tenants" --node-ledger 1 \
  --repeats "$reps" --pod-env "VGPU_LEDGER=1,0" --json-out "$out/ledger.json" --md-out "$out/ledger.md" \
  > "$out/ledger.log" 2>&1
