#!/bin/bash
# Round-4 GPU study (profiles/r4k): do the pods' spinning waits (16 pods in one 16-CPU quota)
# make 16 pods unfair? 16 pods waiting blocked (VGPU_BENCH_SYNC=block, the benchmarks'
# default now) vs spinning (torch's default), then 12 pods blocked; each pod's CPU time in
# the timed window is recorded. lean16: blocked waits plus one OpenMP thread per pod and no
# active wait in the HIP runtime (ROC_ACTIVE_WAIT_TIMEOUT=0), for the start-up's CPU time.
out=${1:-gpurun_out/r4k}
what=${2:-block16,lean16,spin16,block12}
mkdir -p "$out"
if [[ $what == *block16* ]]; then
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --json-out "$out/block16.json" --md-out "$out/block16.md" > "$out/block16.log" 2>&1 || exit $?
fi
if [[ $what == *lean16* ]]; then
  # start-up with one OpenMP thread per pod and no active (spinning) wait in the HIP runtime
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env OMP_NUM_THREADS=1 --pod-env ROC_ACTIVE_WAIT_TIMEOUT=0 --json-out "$out/lean16.json" \
    --md-out "$out/lean16.md" > "$out/lean16.log" 2>&1 || exit $?
fi
if [[ $what == *spin16* ]]; then
  timeout -k 10 380 python -u benchmarks/vgpu_scaling.py --policy default --tenants 16 --seconds 8 \
    --pod-env VGPU_BENCH_SYNC=spin --json-out "$out/spin16.json" --md-out "$out/spin16.md" \
    > "$out/spin16.log" 2>&1 || exit $?
fi
if [[ $what == *block12* ]]; then
  timeout -k 10 300 python -u benchmarks/vgpu_scaling.py --policy default --tenants 12 --seconds 8 \
    --json-out "$out/block12.json" --md-out "$out/block12.md" > "$out/block12.log" 2>&1 || exit $?
fi
