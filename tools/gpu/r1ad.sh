set -o pipefail
# r1ad: whole-sequence LSTM kernel: numerics, suite case 5.1 eager and graph.
OUT=gpurun_out/r1ad; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "lstm" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python benchmarks/aibench_suite.py --cases lstm-inf --steps 20 --warmup 10 \
  --modes native,vgpu,native-graph,vgpu-graph --md-out $OUT/lstm.md > $OUT/lstm.log 2>&1 || { tail -20 $OUT/lstm.log; exit 7; }
cat $OUT/lstm.md
