set -o pipefail
# r1an: row-tile height A/B (BM=64 vs 128) on every ResNet-50 layer; kernel = r1am's LDS epilogue.
OUT=gpurun_out/r1an; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "conv" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
for bm in 64 128; do
  VGPU_CONV_BM=$bm timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv_m$bm.md > $OUT/conv_m$bm.log 2>&1 || { tail -20 $OUT/conv_m$bm.log; exit 7; }
done
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
python3 tools/conv_compare.py $OUT/conv.md $OUT/conv_m64.md $OUT/conv_m128.md
