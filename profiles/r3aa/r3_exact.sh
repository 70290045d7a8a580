#!/bin/bash
# Round-3: the node ledger with exact shares (the plugin sends VGPU_DEVICE_CU_SHARE: 8.3333 %
# at split 12, 6.25 % at split 16), 12 and 16 crowded pods.
#   bash profiles/r3aa/r3_exact.sh <out> [tenants] [repeats]
out=${1:-gpurun_out/r3aa}
tenants=${2:-1,12,16}
reps=${3:-1}
mkdir -p "$out"
timeout -k 10 1080 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants "$tenants" \
  --repeats "$reps" --node-ledger 1 --json-out "$out/exact.json" --md-out "$out/exact.md" > "$out/exact.log" 2>&1
