#!/bin/bash
# Round-4 GPU study (profiles/r4w): DeepLab training b=1 natively, in the suite's
# interception-only pod (ledger on, the default, and off) and in a bare quota vGPU, under
# rocprofv3 with the HIP runtime API traced: GPU busy per step in the timed window and the
# per-function HIP call counts and durations, 2 ABBA runs each.
out=${1:-gpurun_out/r4w}
mkdir -p "$out"
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u tools/probe/prof_tenant.py --out "$out" --case deeplab-train --steps 40 --runs 2 \
  --modes native,vgpu-pod,vgpu-pod-noledger,vgpu-quota --hip-api > "$out/prof.log" 2>&1
echo "prof_rc=$?" >> "$out/prof.log"
