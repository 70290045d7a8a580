#!/bin/bash
# Round-3: bench.py with the node ledger and exact shares for every pod (--ledger).
out=${1:-gpurun_out/r3ac}
mkdir -p "$out"
timeout -k 10 840 python -u bench.py --ledger --json-out "$out/bench.json" > "$out/bench.log" 2>&1
echo "bench_rc=$?" >> "$out/bench.log"
