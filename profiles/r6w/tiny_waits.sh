#!/bin/bash
# Four dispatch-bound pods (tiny kernels, a wait every 8), split-4 vGPUs on the GPU-time
# limiter: the shim's default (polled) wait vs HIP's own, all at once vs pair turns.
set -o pipefail
TAG=${1:-r6w}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
for conc in 0 2; do
  for w in "" native; do
    timeout -k 10 120 python3 benchmarks/tiny_pods.py --pods 4 --conc $conc ${w:+--sync-wait $w} --seconds 4 >> $OUT/tiny.jsonl 2> $OUT/tiny.err \
      || { echo "conc $conc wait ${w:-default} failed"; tail -3 $OUT/tiny.err; exit 1; }
    tail -1 $OUT/tiny.jsonl | python3 -c "import json,sys; d=json.load(sys.stdin); print(d['conc'], d['sync_wait'], d['aggregate_kps'], [p['kps'] for p in d['per_pod']], [p['wait_us'] for p in d['per_pod']])"
  done
done
