#!/bin/bash
# Round-4 GPU study (profiles/r4o): 12 and 16 pods, three times each, with the containers'
# own sampling (default) and with the node ledger's exact charges and shares (--ledger).
out=${1:-gpurun_out/r4o}
mkdir -p "$out"
timeout -k 10 400 python -u bench.py --modes native --sweep on --sweep-tenants 1,12,16,12,16,12,16 \
  --sweep-seconds 8 --time-budget 380 --json-out "$out/default.json" > "$out/default.log" 2>&1 || exit $?
timeout -k 10 400 python -u bench.py --modes native --sweep on --sweep-tenants 1,12,16,12,16,12,16 \
  --sweep-seconds 8 --time-budget 380 --ledger --json-out "$out/ledger.json" > "$out/ledger.log" 2>&1 || exit $?
