set -o pipefail
OUT=gpurun_out/r1e; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_gpu_control.py tests/test_gpu_e2e.py -m gpu -x -q -rs -s -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -8 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/vgpu_scaling.py --solo --policy spatial --tenants 1,2,4,8 --md-out $OUT/solo.md > $OUT/solo.log 2>&1; rc=$?; tail -8 $OUT/solo.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/hook_overhead.py --repeats 2 --md-out $OUT/hooks.md > $OUT/hooks.log 2>&1; rc=$?; grep -E "vGPU stats|\|" $OUT/hooks.log | tail -12; [ $rc -eq 0 ] || exit $rc
