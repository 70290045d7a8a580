# Round-5 GPU study (profiles/r5k, part 8): stock LSTM tenants (4, two per socket; 2 on one
# socket) with their host waits spinning (HIP) vs polled with sleeps by the shim
# (VGPU_SYNC_WAIT=poll), each tenant a quota-only vGPU.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4 --case lstm-inf --shim"
run() {
  local name=$1; shift
  $C "$@" > $O/$name.json 2> $O/$name.err || return $?
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', d['aggregate_items_per_s'], [(t['items_per_s'], t.get('cpus_busy')) for t in d['tenants']])"
}
run w_native_1 --procs 1 --placement local --env VGPU_SYNC_WAIT=native &&
run w_poll_1 --procs 1 --placement local --env VGPU_SYNC_WAIT=poll &&
run w_native_local2 --procs 2 --placement local --env VGPU_SYNC_WAIT=native &&
run w_poll_local2 --procs 2 --placement local --env VGPU_SYNC_WAIT=poll &&
run w_native_split4 --procs 4 --placement split --env VGPU_SYNC_WAIT=native &&
run w_poll_split4 --procs 4 --placement split --env VGPU_SYNC_WAIT=poll &&
run w_auto_split4 --procs 4 --placement split
