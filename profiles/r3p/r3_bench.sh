#!/bin/bash
# Round-3: the driver's default 1-GPU bench run (sweep to 12 pods, node field from the
# sweep's split-4 point), output under $1.
out=${1:-gpurun_out/r3p}
mkdir -p "$out"
timeout -k 10 840 python -u bench.py --json-out "$out/bench.json" > "$out/bench.log" 2>&1
echo "bench_rc=$?" >> "$out/bench.log"
