# Round-5 GPU check, part 4: spilled buffers and CUDA IPC (which placements export), then
# the co-tenancy traces (profiles/r5d).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out
T="python -u -m pytest -v -s --timeout 150 --timeout-method thread -p no:cacheprovider -m gpu"
timeout -k 10 600 $T tests/test_gpu_spill_ipc.py > gpurun_out/g7_ipc.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/g7_ipc.log
grep -E "PASSED|FAILED|passed|failed|AssertionError" gpurun_out/g7_ipc.log
case $rc in 0|1) ;; *) exit $rc ;; esac
bash profiles/r5d/gpu_g5.sh
