#!/bin/bash
# Round-4 GPU check (profiles/r4n): bench.py as the driver runs it (thin-share threshold 40
# CUs), then the steady-state rocprofv3 profile of the headline tenant (timed roctx window).
out=${1:-gpurun_out/r4n}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --json-out "$out/bench.json" > "$out/bench.log" 2>&1 || exit $?
timeout -k 10 500 python -u tools/probe/prof_tenant.py --out "$out/prof" --steps 30 > "$out/prof.log" 2>&1
