# Round-5 GPU check: the whole GPU suite at HEAD, then where a pod's host waits go
# (native vs the shim's polling wait), for the profiles/r5c notes.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g3_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/g3_tests.log
tail -5 gpurun_out/g3_tests.log
[ $rc -eq 0 ] || exit $rc
P="python -u tools/probe/cpu_probe.py --seconds 5"
{
timeout -k 10 120 $P --modes native,vgpu --sync spin --extra-env VGPU_STATS=1 &&
timeout -k 10 120 $P --modes vgpu --sync spin --extra-env VGPU_STATS=1 --extra-env VGPU_SYNC_WAIT=poll &&
timeout -k 10 120 $P --modes vgpu --sync block --extra-env VGPU_STATS=1 &&
timeout -k 10 120 $P --modes vgpu --sync block --extra-env VGPU_STATS=1 --extra-env VGPU_SYNC_WAIT=poll &&
timeout -k 10 120 $P --modes vgpu --sync every --case lstm-inf --extra-env VGPU_STATS=1 &&
timeout -k 10 120 $P --modes vgpu --sync every --case lstm-inf --extra-env VGPU_STATS=1 --extra-env VGPU_SYNC_WAIT=poll
} > gpurun_out/g3_cpu.log 2>&1
rc=$?
cat gpurun_out/g3_cpu.log
exit $rc
