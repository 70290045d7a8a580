#!/bin/bash
# Round-4 GPU study (profiles/r4r): the limiter's credit trace for a lone 25 % pod (solo
# window), and where 16 pods' CPU time goes (per-thread CPU of every pod; MIOpen immediate
# mode so the point starts fast; node ledger on, the plugin's default).
out=${1:-gpurun_out/r4r}
mkdir -p "$out"
timeout -k 10 300 python -u tools/probe/limiter_trace.py --limits 25 --steps 120 --out "$out/trace25.json" \
  > "$out/trace25.log" 2>&1 || exit $?
timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --policy default --tenants 1,16 --seconds 8 \
  --pod-env VGPU_BENCH_AUTOTUNE=0 --json-out "$out/cpu16.json" --md-out "$out/cpu16.md" > "$out/cpu16.log" 2>&1
