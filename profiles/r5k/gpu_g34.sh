# Round-5 GPU study (profiles/r5k, part 3): 3 and 4 LSTM tenants (split over the sockets) with
# HIP's default hardware queues per process and with one - is the slow-down of every kernel
# with four tenants the hardware scheduler running out of queue slots?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5k
mkdir -p $O
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4 --case lstm-inf --placement split"
run() {
  local name=$1; shift
  $C "$@" > $O/$name.json 2> $O/$name.err || return $?
  tail -1 $O/$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', d['aggregate_items_per_s'], [t['items_per_s'] for t in d['tenants']])"
}
run q_default_3 --procs 3 &&
run q_default_4 --procs 4 &&
GPU_MAX_HW_QUEUES=1 run q1_3 --procs 3 &&
GPU_MAX_HW_QUEUES=1 run q1_4 --procs 4 &&
GPU_MAX_HW_QUEUES=1 run q1_8 --procs 8 &&
GPU_MAX_HW_QUEUES=2 run q2_4 --procs 4
