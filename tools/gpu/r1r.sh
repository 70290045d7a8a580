set -o pipefail
# r1r: implicit-GEMM MFMA conv (3x3, strided shortcuts) with fused epilogues: numerics,
# per-layer A/B against MIOpen/CK + epilogue, headline bench A/B, kernel-trace profile.
OUT=gpurun_out/r1r; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
echo "conv tests"
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "conv or resnet50 or stem or prologue" > $OUT/pytest_conv.log 2>&1 || { tail -30 $OUT/pytest_conv.log; exit 6; }
tail -2 $OUT/pytest_conv.log
echo "conv bench"
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md --json-out $OUT/conv.json \
  > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
tail -25 $OUT/conv.log | cut -c1-220
echo "bench A/B"
VGPU_MFMA_CONV=off timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench_off.json \
  > $OUT/bench_off.log 2>&1 || { tail -20 $OUT/bench_off.log; exit 8; }
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench_auto.json \
  > $OUT/bench_auto.log 2>&1 || { tail -20 $OUT/bench_auto.log; exit 9; }
cut -c1-300 $OUT/bench_off.json $OUT/bench_auto.json
echo "profile"
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 10 \
  --modes vgpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 10; }
python3 tools/prof_summary.py "$OUT/prof/**/*results.db" --top 30 -o $OUT/prof_summary.md \
  --title "ResNet-V2-50 inference b=50 bf16 in a vGPU, MFMA convs with fused epilogues (r1r)" > /dev/null || true
ls $OUT/prof | head
