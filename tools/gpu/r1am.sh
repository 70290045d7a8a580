set -o pipefail
# r1am: transposed-product conv with the epilogue on the accumulators (no LDS transpose)
# vs the LDS-transposed epilogue (VGPU_CONV_EPI=lds).
OUT=gpurun_out/r1am; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
VGPU_CONV_EPI=lds timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "conv" > $OUT/pytest_lds.log 2>&1 || { tail -30 $OUT/pytest_lds.log; exit 6; }
tail -1 $OUT/pytest_lds.log
VGPU_CONV_EPI=lds timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv_lds.md > $OUT/conv_lds.log 2>&1 || { tail -20 $OUT/conv_lds.log; exit 7; }
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
python3 tools/conv_compare.py profiles/r1aj/conv.md $OUT/conv_lds.md $OUT/conv.md
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 9; }
cut -c1-200 $OUT/bench.json
