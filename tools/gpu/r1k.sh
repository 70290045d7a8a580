set -o pipefail
OUT=gpurun_out/r1k; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -m pytest tests/test_fused_ops.py -m gpu -x -q -rs -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python benchmarks/aibench_suite.py --steps 20 --warmup 10 --repeats 1 --modes native-graph,vgpu-graph \
  --json-out $OUT/suite_graph.json --md-out $OUT/suite_graph.md > $OUT/suite_graph.log 2>&1; rc=$?; grep -i "failed" $OUT/suite_graph.log | head -5; tail -14 $OUT/suite_graph.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?; tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -m pytest tests/test_gpu_control.py -m gpu -x -q -rs -k priority -p no:cacheprovider > $OUT/pytest_prio.log 2>&1; rc=$?; tail -3 $OUT/pytest_prio.log; [ $rc -eq 0 ] || exit $rc
