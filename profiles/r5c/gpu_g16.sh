# Round-5 GPU study (profiles/r5c, part 2): the 16-pod point's slowest pod with stock waits -
# is the spread from the waits (torch's synchronize every 4 steps vs the harness polling with
# 3 steps in flight) or from the CPU placement (--numa-spread)? 1 + 5 x 16 pods each:
#   spin_nospread  torch's synchronize, VGPU_CPU_SPREAD=0 (pods keep the harness's CPUs)
#   poll_spread    the round-4 harness polling, pods on their vGPU's CPU node (default)
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5c
mkdir -p $out
run() {
  local name=$1; shift
  timeout -k 10 400 python -u bench.py --modes native --sweep on --sweep-tenants 1,16,16,16,16,16 --rccl-probe 0 \
    --time-budget 360 "$@" --json-out "$out/$name.json" > "$out/$name.log" 2>&1
  local rc=$?
  echo "bench_rc=$rc" >> "$out/$name.log"
  python3 -c "import json; d=json.load(open('$out/$name.json')); print('$name', [(p['tenants'], p['aggregate_vs_one'], p['min_tenant_vs_entitlement'], p['cpus_busy']) for p in d['sweep']])"
  return $rc
}
run spin_nospread --sweep-pod-env VGPU_CPU_SPREAD=0 &&
run poll_spread --sweep-pod-env VGPU_BENCH_SYNC=poll
