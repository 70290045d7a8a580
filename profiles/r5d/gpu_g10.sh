# Round-5 GPU study (profiles/r5d, part 2): what serialises two launch-bound processes?
# CPU use per tenant, tenants pinned to cores of their own, one tenant next to CPU-only
# burners, and a HIP API trace of the pair; then the spill/IPC tests again.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
C="timeout -k 10 240 python3 -u tools/probe/cotenancy.py --seconds 4"
run() {  # name, args...
  local name=$1; shift
  $C "$@" > $O/$name.json 2> $O/$name.err || return $?
  tail -1 $O/$name.json | cut -c1-900
}
run cpu_lstm_1 --case lstm-inf --procs 1 &&
run cpu_lstm_2 --case lstm-inf --procs 2 &&
run cpu_lstm_2_pin4 --case lstm-inf --procs 2 --pin 4 &&
run cpu_lstm_1_burn4 --case lstm-inf --procs 1 --burners 4 &&
run cpu_lstm_4 --case lstm-inf --procs 4 &&
run cpu_r152_2_pin4 --case resnet152-inf --procs 2 --pin 4 &&
run hip_lstm_1 --case lstm-inf --procs 1 --trace /tmp/r5d_hip1 --hip-stats &&
python3 tools/probe/cotenancy.py --analyze /tmp/r5d_hip1 > $O/hipoverlap_lstm_1.json &&
run hip_lstm_2 --case lstm-inf --procs 2 --trace /tmp/r5d_hip2 --hip-stats &&
python3 tools/probe/cotenancy.py --analyze /tmp/r5d_hip2 > $O/hipoverlap_lstm_2.json || exit $?
cat $O/hipoverlap_lstm_1.json $O/hipoverlap_lstm_2.json | cut -c1-1500
T="python -u -m pytest -v -s --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 400 $T tests/test_gpu_spill_ipc.py > gpurun_out/g10_ipc.log 2>&1
rc=$?
grep -E "PASSED|FAILED|passed|failed|AssertionError" gpurun_out/g10_ipc.log
exit $rc
