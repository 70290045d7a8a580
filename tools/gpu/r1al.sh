set -o pipefail
# r1al: 3-deep LDS-DMA ring (two K-tiles in flight, counted vmcnt + bare s_barrier) vs 2-deep.
OUT=gpurun_out/r1al; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
VGPU_CONV_STAGES=2 timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv_s2.md > $OUT/conv_s2.log 2>&1 || { tail -20 $OUT/conv_s2.log; exit 7; }
VGPU_CONV_STAGES=3 timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv_s3.md > $OUT/conv_s3.log 2>&1 || { tail -20 $OUT/conv_s3.log; exit 7; }
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
python3 tools/conv_compare.py profiles/r1aj/conv.md $OUT/conv_s2.md $OUT/conv_s3.md $OUT/conv.md
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 9; }
cut -c1-200 $OUT/bench.json
