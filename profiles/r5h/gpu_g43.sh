# Round-5 final check, repeated: the driver's default bench at HEAD (profiles/r5h/bench2.json).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 660 python -u bench.py --json-out gpurun_out/r5h/bench2.json > gpurun_out/r5h/bench2.log 2>&1
rc=$?
tail -1 gpurun_out/r5h/bench2.log | cut -c1-300
python3 -c "
import json; d=json.load(open('gpurun_out/r5h/bench2.json'))
print('value', d.get('value'), 'max_vgpus_per_gpu', d.get('max_vgpus_per_gpu'), 'quota overhead', d.get('overhead_pct_quota_only'))
for p in d.get('sweep', []):
    print(p.get('tenants'), p.get('aggregate_vs_one'), p.get('min_tenant_vs_entitlement'), p.get('cpus_busy'), p.get('skipped', ''))
"
exit $rc
