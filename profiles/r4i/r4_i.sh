#!/bin/bash
# Round-4 GPU study (profiles/r4i): what a pod's first step spends with 1 / 4 / 16 pods starting
# together (CPU time of every pod's threads during start-up, MIOpen's directories). Every pod is
# told the full CU count (VGPU_VIRTUAL_CU_COUNT=0), so all share the lone pod's find-db entries.
out=${1:-gpurun_out/r4i}
mkdir -p "$out"
timeout -k 10 600 python -u benchmarks/vgpu_scaling.py --policy default --tenants 1,4,16 --seconds 5 \
  --pod-env VGPU_VIRTUAL_CU_COUNT=0 --json-out "$out/startup.json" --md-out "$out/startup.md" \
  > "$out/startup.log" 2>&1
rc=$?
{ du -sh ~/.config/miopen ~/.cache/miopen; find ~/.config/miopen ~/.cache/miopen -maxdepth 3 | head -40; } \
  > "$out/miopen_dirs.txt" 2>&1
nproc > "$out/cpus.txt"; cat /sys/fs/cgroup/cpu.max >> "$out/cpus.txt" 2>/dev/null
exit $rc
