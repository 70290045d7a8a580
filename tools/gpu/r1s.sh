set -o pipefail
# r1s: stem kernel with batched staging loads; bench + steady-state profile.
OUT=gpurun_out/r1s; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "stem or resnet50 or prologue" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md --json-out $OUT/conv.json \
  > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
grep -E "stem|sum" $OUT/conv.md
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 \
  || { tail -20 $OUT/bench.log; exit 9; }
cut -c1-200 $OUT/bench.json
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 20 --warmup 10 \
  --modes vgpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 10; }
python3 tools/prof_summary.py "$OUT/prof/**/*results.db" --after-last naive_conv --top 30 -o $OUT/prof_ss.md \
  --title "ResNet-V2-50 inference b=50 bf16 in a vGPU, steady state (r1s)" > /dev/null || true
