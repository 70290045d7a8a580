#!/bin/bash
# Launch-bound co-tenancy, third pass: is it the number of processes with
# work in flight, or with queues mapped at all? Active tiny-kernel processes next to idle ones
# (HIP initialised, a stream's queue created and used, then asleep through the window); three
# active processes repeated (one of them ran at full speed in r6f); four processes with one
# hardware queue each. All pinned to cores of one NUMA node, HIP's spinning wait.
set -o pipefail
TAG=${1:-r6f3}; SECS=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
P=4paradigm-k8s-device-plugin_amd/lib/cotenancy_probe
run() {
  timeout -k 10 60 $P "$@" >> $OUT/idle.jsonl 2>> $OUT/idle.err || { echo "$* failed rc=$?"; exit 1; }
  tail -1 $OUT/idle.jsonl | python3 -c "
import json,sys; d=json.load(sys.stdin); t=d['per_tenant']
print(d['mode'], d['tenants'], 'idle', d['idle'], d['wait'], d['pin'], round(d['aggregate_kps']), [round(x['kps']/1e3,1) for x in t],
      'wait_us', [round(x['wait_us'],1) for x in t], 'p90', max(x['p90_us'] for x in t))"
}
run procs 1 $SECS 5 4 spin same 0
run procs 1 $SECS 5 4 spin same 1
run procs 1 $SECS 5 4 spin same 3
run procs 2 $SECS 5 4 spin same 0
run procs 2 $SECS 5 4 spin same 1
run procs 2 $SECS 5 4 spin same 2
run procs 2 $SECS 5 4 spin same 6
for r in 1 2 3; do run procs 3 $SECS 5 4 spin same 0; done
GPU_MAX_HW_QUEUES=1 run procs 4 $SECS 5 4 spin same 0
run procs 4 $SECS 5 32 spin same 0
run procs 4 $SECS 50 4 spin same 0
