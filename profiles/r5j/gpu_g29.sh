# Round-5 final check, repeated at the end of the round: the whole GPU suite at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5j
timeout -k 10 1100 python -u -m pytest tests -m gpu -v --timeout 300 --timeout-method thread -p no:cacheprovider \
  > gpurun_out/r5j/gpu_tests.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/r5j/gpu_tests.log
grep -E "FAILED|ERROR|passed|failed" gpurun_out/r5j/gpu_tests.log | tail -15
exit $rc
