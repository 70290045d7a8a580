# Round-5 GPU study (profiles/r5d, part 4): does the same-socket serialisation of two
# launch-bound tenants come from the per-launch read-back of kernel arguments that HIP writes
# into device memory (HIP_FORCE_DEV_KERNARG=1, its MI300/MI355X default)? The same placements
# with kernel arguments in host memory; then the spill/IPC tests.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4"
run() {  # name, args...
  local name=$1; shift
  $C "$@" > $O/$name.json 2> $O/$name.err || return $?
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', d['aggregate_items_per_s'], [(t['items_per_s'], t.get('numa_seen'), t.get('cpus_busy')) for t in d['tenants']])"
}
for k in 0 1; do
  export HIP_FORCE_DEV_KERNARG=$k
  run ka${k}_lstm-inf_local1 --case lstm-inf --procs 1 --placement local &&
  run ka${k}_lstm-inf_local2 --case lstm-inf --procs 2 --placement local &&
  run ka${k}_lstm-inf_remote2 --case lstm-inf --procs 2 --placement remote &&
  run ka${k}_resnet152-inf_local1 --case resnet152-inf --procs 1 --placement local &&
  run ka${k}_resnet152-inf_local2 --case resnet152-inf --procs 2 --placement local &&
  run ka${k}_resnet50-inf_local1 --case resnet50-inf --procs 1 --placement local || exit $?
done
unset HIP_FORCE_DEV_KERNARG
T="python -u -m pytest -v -s --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 400 $T tests/test_gpu_spill_ipc.py > gpurun_out/g12_ipc.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|^E " gpurun_out/g12_ipc.log | cut -c1-400
exit $rc
