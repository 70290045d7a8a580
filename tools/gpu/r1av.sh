set -o pipefail
# r1av: re-validation after the container re-creation: full GPU test suite, smoke, headline bench.
OUT=gpurun_out/r1av; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
echo "pytest gpu"
timeout -k 10 840 python -u -m pytest tests -m gpu -v -rs -x -p no:cacheprovider --timeout 300 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1 || { tail -30 $OUT/pytest_gpu.log; exit 2; }
tail -3 $OUT/pytest_gpu.log
echo "smoke"
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 3; }
tail -2 $OUT/smoke.log
echo "bench"
timeout -k 10 240 python bench.py --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 4; }
cut -c1-220 $OUT/bench.json
