#!/bin/bash
# Launch-bound co-tenancy, pinned (second pass): the tiny-kernel probe as N
# processes vs N threads of one process, every tenant pinned to a physical core of one NUMA node
# ("same") or alternating nodes ("split"), with HIP's spinning wait, a blocking (interrupt) wait
# or a polled hipStreamQuery. Per tenant: kernels/s, in-kernel duration, host time per launch
# call and per wait. One JSON line per run into gpurun_out/<tag>/pin.jsonl.
set -o pipefail
TAG=${1:-r6f2}; SECS=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
P=4paradigm-k8s-device-plugin_amd/lib/cotenancy_probe
run() {
  timeout -k 10 60 $P "$@" >> $OUT/pin.jsonl 2>> $OUT/pin.err || { echo "$* failed rc=$?"; exit 1; }
  tail -1 $OUT/pin.jsonl | python3 -c "
import json,sys; d=json.load(sys.stdin); t=d['per_tenant']
print(d['mode'], d['tenants'], d['wait'], d['pin'], round(d['aggregate_kps']), [round(x['kps']/1e3,1) for x in t],
      'launch_us', [round(x['launch_us'],2) for x in t], 'wait_us', [round(x['wait_us'],1) for x in t],
      'nodes', [x['node'] for x in t], 'p90', max(x['p90_us'] for x in t))"
}
for w in spin poll block; do run procs 1 $SECS 5 4 $w same; done
for n in 2 4; do
  for w in spin poll block; do
    for pin in same split; do
      for mode in procs streams; do run $mode $n $SECS 5 4 $w $pin; done
    done
  done
done
