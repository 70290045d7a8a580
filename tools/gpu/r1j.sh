set -o pipefail
OUT=gpurun_out/r1j; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_fused_ops.py tests/test_gpu_shim.py -m gpu -x -q -rs -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/op_bench.py --md-out $OUT/op_bench.md > $OUT/op_bench.log 2>&1; rc=$?; tail -8 $OUT/op_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 700 python benchmarks/aibench_suite.py --cases lstm-inf,lstm-train,deeplab-inf,resnet50-inf --steps 20 --warmup 10 --repeats 2 \
  --modes native,vgpu,vgpu-nolaunch,vgpu-stats,native-graph,vgpu-graph --md-out $OUT/suite_diag.md > $OUT/suite_diag.log 2>&1; rc=$?
grep "vGPU stats" $OUT/suite_diag.log | head -2; tail -8 $OUT/suite_diag.log; [ $rc -eq 0 ] || exit $rc
