#!/bin/bash
# Round-3: the node ledger with shares that add up to at most the whole GPU. The ledger's
# charges come from one snapshot, so they add up to at most the GPU's busy time; with the
# plugin's rounded-up shares (12 x 9 % = 108 %, 16 x 7 % = 112 %) the limiter then never
# binds in aggregate (profiles/r3v). Here 12 x 8 % and 16 x 6 % (96 %), ledger on.
out=${1:-gpurun_out/r3w}
mkdir -p "$out"
timeout -k 10 500 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants 1,12 --node-ledger 1 \
  --pod-env VGPU_DEVICE_CU_LIMIT_0=8 --json-out "$out/l12.json" --md-out "$out/l12.md" > "$out/l12.log" 2>&1
rc=$?
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --policy default --seconds 10 --tenants 16 --node-ledger 1 \
  --pod-env VGPU_DEVICE_CU_LIMIT_0=6 --json-out "$out/l16.json" --md-out "$out/l16.md" > "$out/l16.log" 2>&1
