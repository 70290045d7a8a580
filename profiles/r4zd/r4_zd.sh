#!/bin/bash
# Round-4 GPU study (profiles/r4zd): the 16-pod point four times, with HIP's default hardware
# queues per pod and with one (GPU_MAX_HW_QUEUES=1: 16 user queues instead of ~70 on the
# GPU's hardware queue slots), polling waits, common-window rating.
out=${1:-gpurun_out/r4zd}
mkdir -p "$out"
for q in default 1; do
  extra=""
  [ "$q" = default ] || extra="--sweep-pod-env GPU_MAX_HW_QUEUES=$q"
  timeout -k 10 420 python -u bench.py --modes native --sweep on --sweep-tenants 1,16,16,16,16 --rccl-probe 0 \
    --time-budget 380 $extra --json-out "$out/q$q.json" > "$out/q$q.log" 2>&1
  rc=$?
  echo "bench_rc=$rc" >> "$out/q$q.log"
  [ $rc -eq 0 ] || exit $rc
done
