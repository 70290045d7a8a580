set -o pipefail
# r1au: full GPU test suite, smoke, headline bench, 10-case suite (eager and HIP-graph) after the
# LDS-DMA conv kernel, dual-source projection GEMM and fragment prologue.
OUT=gpurun_out/r1au; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
echo "pytest gpu"
timeout -k 10 1200 python -u -m pytest tests -m gpu -q -rs -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -3 $OUT/pytest_gpu.log
echo "smoke"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -2 $OUT/smoke.log
echo "bench"
timeout -k 10 600 python bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 4; }
cut -c1-220 $OUT/bench.json
echo "suite"
timeout -k 10 1200 python benchmarks/aibench_suite.py --steps 20 --warmup 10 --repeats 2 --modes native,vgpu \
  --json-out $OUT/suite.json --md-out $OUT/suite.md > $OUT/suite.log 2>&1 || { tail -20 $OUT/suite.log; exit 5; }
cat $OUT/suite.md
timeout -k 10 900 python benchmarks/aibench_suite.py --steps 20 --warmup 10 --repeats 1 --modes native-graph,vgpu-graph \
  --json-out $OUT/suite_graph.json --md-out $OUT/suite_graph.md > $OUT/suite_graph.log 2>&1 || { tail -20 $OUT/suite_graph.log; exit 6; }
cat $OUT/suite_graph.md
