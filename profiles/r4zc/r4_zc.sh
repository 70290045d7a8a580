#!/bin/bash
# Round-4 bench check (profiles/r4zc): bench.py as the driver runs it, with the sweep's pods
# waiting by polling (3 steps in flight, sleeping between event queries) instead of HIP's
# blocking event wait, which keeps a CPU busy (profiles/r4za).
out=${1:-gpurun_out/r4zc}
mkdir -p "$out"
timeout -k 10 700 python -u bench.py --json-out "$out/bench.json" > "$out/bench.log" 2>&1
echo "bench_rc=$?" >> "$out/bench.log"
