# Round-5 GPU study (profiles/r5c, part 5): as part 4, with each pod's charged processes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 400 python -u bench.py --modes native --sweep on --sweep-tenants 1,16,16,16 --rccl-probe 0 \
  --time-budget 360 --json-out "$out/diag16b.json" > "$out/diag16b.log" 2>&1
rc=$?
python3 -c "
import json; d=json.load(open('$out/diag16b.json'))
for p in d['sweep']:
    if p['tenants'] != 16: continue
    t = p['per_tenant']; i = min(range(16), key=lambda k: t[k])
    print(round(p['min_tenant_vs_entitlement'], 3), 'slowest', i, p['region_procs'][i], 'pod0', p['region_procs'][0], 'pod5', p['region_procs'][5])
"
exit $rc
