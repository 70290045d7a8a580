#!/bin/bash
# Round-4 bench check (profiles/r4x): bench.py as the driver runs it, with concurrent pods
# rated over the window in which all of them run (bench.common_window).
out=${1:-gpurun_out/r4x}
mkdir -p "$out"
timeout -k 10 700 python -u bench.py --json-out "$out/bench.json" > "$out/bench.log" 2>&1
echo "bench_rc=$?" >> "$out/bench.log"
