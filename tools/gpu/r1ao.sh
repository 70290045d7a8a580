set -o pipefail
# r1ao: projection blocks' conv3 + shortcut as one dual-source GEMM (conv_dual).
OUT=gpurun_out/r1ao; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
tail -8 $OUT/conv.md
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 9; }
cut -c1-300 $OUT/bench.json
