# Round-5 GPU run (profiles/r5c, part 7): the default configuration (stock waits, queue bound
# 16, NUMA spread) at 12 and 16 pods, three points each.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
timeout -k 10 500 python -u bench.py --modes native --sweep on --sweep-tenants 1,12,12,12,16,16,16 --rccl-probe 0 \
  --time-budget 460 --json-out "$out/default_12_16.json" > "$out/default_12_16.log" 2>&1
rc=$?
echo "bench_rc=$rc" >> "$out/default_12_16.log"
python3 -c "import json; d=json.load(open('$out/default_12_16.json')); print([(p['tenants'], p.get('aggregate_vs_one'), p.get('min_tenant_vs_entitlement'), p.get('cpus_busy'), p.get('skipped','')) for p in d['sweep']])"
exit $rc
