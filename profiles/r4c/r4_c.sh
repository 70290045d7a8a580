#!/bin/bash
# Round-4 GPU study 3 (profiles/r4c):
#   lone   a lone ResNet-50 b=50 pod at 25 % on the GPU-time limiter: solo window off /
#          160 ms (default) / 320 ms (achieved share of native throughput, charged share)
#   many   16 pods: start-up phases (bench sweep 1,16); then 16 pods told the GPU's full CU
#          count (VGPU_VIRTUAL_CU_COUNT=0: crowded pods run on all CUs, so libraries should
#          size for 256, not the 16 of their slice); then the board's concurrency
#          admission at 1 (time slicing) for the per-pod spread
# Each GPU step has its own time limit; a crash/timeout ends the script.
out=${1:-gpurun_out/r4c}
what=${2:-lone,sweep,fullcu,conc1}
mkdir -p "$out"
# The hardware scheduler's limits: processes mapped at once (one VMID each) and its policy.
for f in hws_max_conc_proc sched_policy hws_gws_support mes sched_hw_submission; do
  echo "$f=$(cat /sys/module/amdgpu/parameters/$f 2>/dev/null)"
done > "$out/hws.txt"
if [[ $what == *lone* ]]; then
  for w in 0 160 320; do
    timeout -k 10 240 python -u benchmarks/temporal_accuracy.py --workload resnet50 --tenants 1 --limits 25 \
      --seconds 8 --extra VGPU_LIMITER_SOLO_WINDOW_MS=$w --json-out "$out/lone_w$w.json" --md-out "$out/lone_w$w.md" \
      > "$out/lone_w$w.log" 2>&1 || exit $?
  done
fi
if [[ $what == *sweep* ]]; then
  timeout -k 10 560 python -u bench.py --modes native --sweep on --sweep-tenants 1,16 --sweep-seconds 8 \
    --time-budget 520 --json-out "$out/sweep16.json" > "$out/sweep16.log" 2>&1 || exit $?
fi
if [[ $what == *fullcu* ]]; then
  timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_VIRTUAL_CU_COUNT=0 --json-out "$out/fullcu_16.json" --md-out "$out/fullcu_16.md" \
    > "$out/fullcu_16.log" 2>&1 || exit $?
fi
if [[ $what == *conc8* ]]; then
  timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_GPU_CONCURRENCY=8 --json-out "$out/conc8_16.json" --md-out "$out/conc8_16.md" \
    > "$out/conc8_16.log" 2>&1 || exit $?
fi
if [[ $what == *conc1* ]]; then
  timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_GPU_CONCURRENCY=1 --json-out "$out/conc1_16.json" --md-out "$out/conc1_16.md" \
    > "$out/conc1_16.log" 2>&1 || exit $?
fi
