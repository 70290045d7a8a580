#!/bin/bash
# Round-4 GPU check (profiles/r4m): bench.py exactly as the driver runs it on one GPU.
out=${1:-gpurun_out/r4m}
mkdir -p "$out"
timeout -k 10 600 python -u bench.py --json-out "$out/bench.json" > "$out/bench.log" 2>&1
echo "bench_rc=$?" >> "$out/bench.log"
