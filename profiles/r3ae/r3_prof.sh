#!/bin/bash
# Round-3: rocprofv3 kernel traces of the headline tenant at HEAD (native, quota-only vGPU,
# 25 % temporal vGPU with the shim's roctx ranges), summaries under $1.
out=${1:-gpurun_out/r3ae}
mkdir -p "$out"
export TMPDIR=/tmp
timeout -k 10 700 python -u tools/probe/prof_tenant.py --out "$out/prof" > "$out/prof.log" 2>&1
