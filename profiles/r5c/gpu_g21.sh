# Round-5 GPU study (profiles/r5c, part 6): the 16-pod point with stock waits and a bounded
# queue on the limiter (VGPU_CROWD_DEPTH=16 vs 64), A B A B on one box.
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
run depth16_a --sweep-pod-env VGPU_CROWD_DEPTH=16 && run depth64_c --sweep-pod-env VGPU_CROWD_DEPTH=64 &&
run depth16_b --sweep-pod-env VGPU_CROWD_DEPTH=16 && run depth64_d --sweep-pod-env VGPU_CROWD_DEPTH=64
