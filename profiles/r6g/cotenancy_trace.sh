#!/bin/bash
# Which host call carries the per-socket effect? Two stock LSTM inference
# tenants (no shim), both on the GPU's socket ("local") vs one per socket ("split"):
#   1. plain runs (no profiler): the effect itself, today;
#   2. each tenant under its own rocprofv3 --kernel-trace --hip-trace --hsa-trace --stats,
#      analysed into per-tenant kernel overlap plus the HIP and HSA calls that took the most
#      time. The big per-call trace CSVs are removed afterwards (the stats stay).
set -o pipefail
TAG=${1:-r6g}; SECS=${2:-3}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
P=tools/probe/cotenancy.py
for pl in local split; do
  timeout -k 10 300 python3 $P --case lstm-inf --procs 2 --seconds 6 --placement $pl > $OUT/plain_$pl.json 2> $OUT/plain_$pl.err \
    || { echo "plain $pl failed"; tail -5 $OUT/plain_$pl.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('plain', sys.argv[2], d['aggregate_items_per_s'], [t['items_per_s'] for t in d['tenants']])" $OUT/plain_$pl.json $pl
done
timeout -k 10 120 python3 $P --case lstm-inf --procs 1 --seconds 6 --placement local > $OUT/plain_one.json 2> $OUT/plain_one.err \
  || { echo "plain one failed"; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('plain one', d['aggregate_items_per_s'])" $OUT/plain_one.json
for pl in one local split; do
  n=2; [ $pl = one ] && n=1
  ppl=$pl; [ $pl = one ] && ppl=local
  timeout -k 10 400 python3 $P --case lstm-inf --procs $n --seconds $SECS --placement $ppl --trace $OUT/tr_$pl --hip-stats --hsa-stats \
    > $OUT/traced_$pl.json 2> $OUT/traced_$pl.err || { echo "traced $pl failed"; tail -5 $OUT/traced_$pl.err; exit 1; }
  python3 $P --analyze $OUT/tr_$pl > $OUT/analysis_$pl.json || exit 1
  find $OUT/tr_$pl -name '*_trace.csv' -delete
  du -sh $OUT/tr_$pl
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1])); t=json.load(open(sys.argv[2]))
print('traced', sys.argv[3], t['aggregate_items_per_s'], 'any', d.get('any'), 'both', d.get('both'))
for api in ('hip_api','hsa_api'):
    for ten, rows in sorted(d.get(api, {}).items()):
        print(' ', api, ten, [(r['api'], r['calls'], r['avg_us']) for r in rows[:4]])
" $OUT/analysis_$pl.json $OUT/traced_$pl.json $pl
done
