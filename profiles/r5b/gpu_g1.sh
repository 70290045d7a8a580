set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 1080 python -u -m pytest tests -m gpu -x -v -k "not deepbind" --timeout 300 --timeout-method thread -p no:cacheprovider > gpurun_out/g1_tests.log 2>&1
echo "pytest rc=$?" >> gpurun_out/g1_tests.log
tail -40 gpurun_out/g1_tests.log
