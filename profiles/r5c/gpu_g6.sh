# Round-5 GPU check, part 3: spilled buffers over IPC / RCCL, the background-class test twice
# (with the limiter's diagnostics), then where a pod's host waits go (native vs polling).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -v -s --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 600 $T tests/test_gpu_spill_ipc.py > gpurun_out/g6_ipc.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/g6_ipc.log
grep -E "PASSED|FAILED|passed|failed|RESULT" gpurun_out/g6_ipc.log
case $rc in 0|1) ;; *) exit $rc ;; esac
for i in 1 2; do
  timeout -k 10 300 $T "tests/test_gpu_limits.py::test_background_class_yields_to_a_busy_latency_class" > gpurun_out/g6_bg$i.log 2>&1
  rc=$?
  grep -E "next_to_equal|PASSED|FAILED" gpurun_out/g6_bg$i.log
  case $rc in 0|1) ;; *) exit $rc ;; esac
done
P="python -u tools/probe/cpu_probe.py --seconds 5"
for args in "--modes native,vgpu --sync spin" "--modes vgpu --sync spin --extra-env VGPU_SYNC_WAIT=poll" \
            "--modes vgpu --sync block" "--modes vgpu --sync block --extra-env VGPU_SYNC_WAIT=poll" \
            "--modes native,vgpu --sync every --case lstm-inf" "--modes vgpu --sync every --case lstm-inf --extra-env VGPU_SYNC_WAIT=poll"; do
  echo "== $args" >> gpurun_out/g6_cpu.log
  timeout -k 10 150 $P $args --extra-env VGPU_STATS=1 >> gpurun_out/g6_cpu.log 2>&1 || exit $?
  tail -3 gpurun_out/g6_cpu.log
done
