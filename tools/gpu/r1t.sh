set -o pipefail
# r1t: A/B of the conv kernel's register pipeline depth (libvgpu_ops.so vs libvgpu_ops_deep.so).
OUT=gpurun_out/r1t; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
VGPU_OPS_LIB=libvgpu_ops_deep.so timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -v --timeout 120 \
  --timeout-method thread -p no:cacheprovider -k "conv or prologue" > $OUT/pytest_deep.log 2>&1 \
  || { tail -30 $OUT/pytest_deep.log; exit 6; }
tail -1 $OUT/pytest_deep.log
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
VGPU_OPS_LIB=libvgpu_ops_deep.so timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv_deep.md \
  > $OUT/conv_deep.log 2>&1 || { tail -20 $OUT/conv_deep.log; exit 8; }
paste -d'\n' <(cut -d'|' -f2,7 $OUT/conv.md) <(cut -d'|' -f2,7 $OUT/conv_deep.md) | head -60
