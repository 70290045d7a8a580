# Round-5 GPU study (profiles/r5d, part 8): is the same-socket serialisation of two PyTorch
# launch-bound tenants carried by ROCr's interrupt-driven signal waits? The same LSTM pairs
# with HSA_ENABLE_INTERRUPT=0 (ROCr polls its signals instead of sleeping in KFD events).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4 --case lstm-inf"
run() {
  local name=$1; shift
  $C "$@" > $O/$name.json 2> $O/$name.err || return $?
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', d['aggregate_items_per_s'], [(t['items_per_s'], t.get('cpus_busy')) for t in d['tenants']])"
}
export HSA_ENABLE_INTERRUPT=0
run noint_local1 --procs 1 --placement local &&
run noint_local2 --procs 2 --placement local &&
run noint_split2 --procs 2 --placement split &&
run noint_local4 --procs 4 --placement local &&
run noint_split4 --procs 4 --placement split || exit $?
unset HSA_ENABLE_INTERRUPT
run int_split4 --procs 4 --placement split
