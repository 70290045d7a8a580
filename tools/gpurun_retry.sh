#!/bin/bash
# Retries a gpurun call while no box is free (status=transient: nothing ran, nothing charged).
# A call that ran - passed or failed - is never repeated.
#   tools/gpurun_retry.sh <out-file> <timeout-s> <command>
out=$1; to=$2; cmd=$3
for i in $(seq 1 30); do
  /usr/local/graft/bin/gpurun --timeout "$to" -- "$cmd" > "$out" 2>&1
  grep -q "status=transient" "$out" || exit 0
  sleep 90
done
