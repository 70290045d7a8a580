# Round-5 checks: the background-class test (reworked), then the suite's noisy VGG-16
# training case (profiles/r5f).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_limits.py::test_background_class_yields_to_a_busy_latency_class" > gpurun_out/r5h/bg_test2.log 2>&1
rc=$?
grep -E "next_to_equal|PASSED|FAILED" gpurun_out/r5h/bg_test2.log | cut -c1-600
case $rc in 0|1) ;; *) exit $rc ;; esac
bash tools/gpu_g9.sh vgg16-train
