# Round-5 GPU study (profiles/r5c, part 3): the 16-pod point with stock waits, --numa-spread
# on (default) vs off (VGPU_CPU_SPREAD=0), alternated A B A B on one box; every point records
# each pod's GPU time charged by its limiter (granted_pct).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --modes native --sweep on --sweep-tenants 1,16,16,16,16 --rccl-probe 0 \
    --time-budget 360 "$@" --json-out "$out/$name.json" > "$out/$name.log" 2>&1
  local rc=$?
  echo "bench_rc=$rc" >> "$out/$name.log"
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', [(p['tenants'], p['aggregate_vs_one'], p['min_tenant_vs_entitlement'], p['cpus_busy']) for p in d['sweep']])"
  return $rc
}
run ab_spread1 && run ab_nospread1 --sweep-pod-env VGPU_CPU_SPREAD=0 &&
run ab_spread2 && run ab_nospread2 --sweep-pod-env VGPU_CPU_SPREAD=0
