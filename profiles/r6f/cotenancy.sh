#!/bin/bash
# Launch-bound co-tenancy mechanism: the same tiny kernels as N processes
# vs N streams of one process (native/tests/cotenancy_probe.hip), no shim. One JSON line per run
# into gpurun_out/<tag>/cotenancy.jsonl.
set -o pipefail
TAG=${1:-r6f}; SPIN=${2:-5}; GRID=${3:-4}; SECS=${4:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
P=4paradigm-k8s-device-plugin_amd/lib/cotenancy_probe
for n in 1 2 3 4 8; do
  for mode in procs streams; do
    timeout -k 10 60 $P $mode $n $SECS $SPIN $GRID >> $OUT/cotenancy.jsonl 2>> $OUT/cotenancy.err || { echo "$mode $n failed rc=$?"; exit 1; }
    tail -1 $OUT/cotenancy.jsonl | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['mode'], d['tenants'], round(d['aggregate_kps']), [round(t['p50_us'],1) for t in d['per_tenant']], [round(t['p90_us'],1) for t in d['per_tenant']], d['amdgpu'])"
  done
done
