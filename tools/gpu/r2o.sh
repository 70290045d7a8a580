#!/bin/bash
# Round 2o: limiter trace (granted vs charged per step) for the bench tenant.
out=gpurun_out/r2o; mkdir -p $out
step() {
  local name=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $out/$name.log 2>&1; local rc=$?
  echo "$name rc=$rc" >> $out/steps.txt
  if [ $rc -ne 0 ]; then exit $rc; fi
}
step trace_nosync 400 python -u tools/probe/limiter_trace.py --limits 99,50,25,10 --steps 60 --out $out/trace_nosync.json
step trace_sync4 400 python -u tools/probe/limiter_trace.py --limits 99,25 --steps 60 --sync-every 4 --out $out/trace_sync4.json
