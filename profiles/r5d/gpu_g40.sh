# Round-5 GPU study (profiles/r5d, part 9): two stock LSTM tenants on one socket (1.00x) with
# CLR's signal / wait / kernel-argument knobs changed one at a time - which runtime path
# carries the per-socket effect?
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
C="timeout -k 5 90 python3 -u tools/probe/cotenancy.py --seconds 4 --case lstm-inf --procs 2 --placement local"
run() {
  local name=$1; shift
  env "$@" $C > $O/knob_$name.json 2> $O/knob_$name.err || return $?
  tail -1 $O/knob_$name.json | python3 -c "import json,sys; d=json.load(sys.stdin); print('$name', d['aggregate_items_per_s'], [t['items_per_s'] for t in d['tenants']])"
}
# (ROC_SYSTEM_SCOPE_SIGNAL=0 hangs the tenants: their waits never see the GPU's signal
# updates - first attempt of this script)
run activewait0 ROC_ACTIVE_WAIT_TIMEOUT=0 &&
run cpuwait1 ROC_CPU_WAIT_FOR_SIGNAL=1 &&
run cpuwait0 ROC_CPU_WAIT_FOR_SIGNAL=0 &&
run fgskernarg0 ROC_USE_FGS_KERNARG=0 &&
run fgskernarg1 ROC_USE_FGS_KERNARG=1
