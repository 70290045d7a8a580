# Round-5 GPU study (profiles/r5d, part 3): two launch-bound tenants by CPU placement - both on
# the GPU's NUMA node, both on another node, one on each - and unpinned (where they ran), for
# LSTM inference and ResNet-152 b=10; then the spill/IPC tests again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4"
run() {  # name, args...
  local name=$1; shift
  $C "$@" > $O/$name.json 2> $O/$name.err || return $?
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', d['aggregate_items_per_s'], d.get('gpu_numa_node'), d.get('numa_cpus'), [(t['items_per_s'], t.get('numa_seen'), t.get('cpu_last')) for t in d['tenants']])"
}
for c in lstm-inf resnet152-inf; do
  run pl_${c}_local1 --case $c --procs 1 --placement local &&
  run pl_${c}_remote1 --case $c --procs 1 --placement remote &&
  run pl_${c}_local2 --case $c --procs 2 --placement local &&
  run pl_${c}_remote2 --case $c --procs 2 --placement remote &&
  run pl_${c}_split2 --case $c --procs 2 --placement split &&
  run pl_${c}_none2a --case $c --procs 2 &&
  run pl_${c}_none2b --case $c --procs 2 || exit $?
done
run pl_lstm-inf_local4 --case lstm-inf --procs 4 --placement local || exit $?
T="python -u -m pytest -v -s --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 400 $T tests/test_gpu_spill_ipc.py > gpurun_out/g11_ipc.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/g11_ipc.log | cut -c1-400
exit $rc
