# Round-5 GPU study (profiles/r5c, part 4): 16 pods with stock waits, per pod the GPU time its
# limiter charged and the time its launches waited at the gate - why one pod falls behind.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 400 python -u bench.py --modes native --sweep on --sweep-tenants 1,16,16,16,16 --rccl-probe 0 \
  --time-budget 360 --json-out "$out/diag16.json" > "$out/diag16.log" 2>&1
rc=$?
python3 -c "
import json; d=json.load(open('$out/diag16.json'))
for p in d['sweep']:
    if p['tenants'] != 16: continue
    t = p['per_tenant']; i = min(range(16), key=lambda k: t[k])
    print(round(p['min_tenant_vs_entitlement'], 3), 'slowest', i, 'granted', p['granted_pct'][i], 'throttled', p['throttled_pct'][i],
          'others granted', sorted(p['granted_pct'])[8], 'throttled', sorted(p['throttled_pct'])[8])
"
exit $rc
