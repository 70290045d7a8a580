# Round-5 GPU check, part 2: why the background class stopped yielding (bg_yield probe),
# the rest of the GPU suite after test_gpu_limits' background test, the spill/IPC tests,
# then where a pod's host waits go (native vs the shim's polling wait).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 150 python -u tools/probe/bg_yield.py --neighbour-prio 0 > gpurun_out/g4_bgy0.log 2>&1 &&
timeout -k 10 150 python -u tools/probe/bg_yield.py --neighbour-prio 2 > gpurun_out/g4_bgy2.log 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest tests/test_gpu_limits.py tests/test_gpu_overhead.py tests/test_gpu_shim.py \
  tests/test_gpu_spill_ipc.py -m gpu -v --maxfail 4 --timeout 300 --timeout-method thread -p no:cacheprovider \
  --deselect tests/test_gpu_limits.py::test_background_class_yields_to_a_busy_latency_class \
  -k "not temporal_accuracy_single and not through_the_node_ledger and not two_tenants_stock and not lone_pod and not four_light" \
  > gpurun_out/g4_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/g4_tests.log
tail -5 gpurun_out/g4_tests.log
case $rc in 0|1) ;; *) exit $rc ;; esac
P="python -u tools/probe/cpu_probe.py --seconds 5"
{
timeout -k 10 120 $P --modes native,vgpu --sync spin --extra-env VGPU_STATS=1 &&
timeout -k 10 120 $P --modes vgpu --sync spin --extra-env VGPU_STATS=1 --extra-env VGPU_SYNC_WAIT=poll &&
timeout -k 10 120 $P --modes vgpu --sync block --extra-env VGPU_STATS=1 &&
timeout -k 10 120 $P --modes vgpu --sync block --extra-env VGPU_STATS=1 --extra-env VGPU_SYNC_WAIT=poll &&
timeout -k 10 120 $P --modes vgpu --sync every --case lstm-inf --extra-env VGPU_STATS=1 &&
timeout -k 10 120 $P --modes vgpu --sync every --case lstm-inf --extra-env VGPU_STATS=1 --extra-env VGPU_SYNC_WAIT=poll
} > gpurun_out/g4_cpu.log 2>&1
rc2=$?
tail -30 gpurun_out/g4_cpu.log
[ $rc2 -eq 0 ] && exit $rc
exit $rc2
