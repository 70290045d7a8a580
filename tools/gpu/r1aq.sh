set -o pipefail
# r1aq: cache policy of the conv epilogue (nontemporal residual loads / output stores), and
# the headline step without the dead sum output before dual projection blocks.
OUT=gpurun_out/r1aq; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "resnet or dual" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
for v in "" _rt _ynt _both; do
  VGPU_OPS_LIB=libvgpu_ops$v.so timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv$v.md > $OUT/conv$v.log 2>&1 || { tail -20 $OUT/conv$v.log; exit 7; }
done
python3 tools/conv_compare.py $OUT/conv.md $OUT/conv_rt.md $OUT/conv_ynt.md $OUT/conv_both.md
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 9; }
cut -c1-200 $OUT/bench.json
