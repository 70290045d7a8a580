set -o pipefail
# r1v: VGG-16 inference on the MFMA conv kernel (bias + ReLU epilogue).
OUT=gpurun_out/r1v; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "vgg" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
VGPU_MFMA_CONV=off timeout -k 10 600 python benchmarks/aibench_suite.py --cases vgg16-inf --steps 20 --warmup 10 \
  --modes native,vgpu --md-out $OUT/vgg_off.md > $OUT/vgg_off.log 2>&1 || { tail -20 $OUT/vgg_off.log; exit 7; }
timeout -k 10 600 python benchmarks/aibench_suite.py --cases vgg16-inf --steps 20 --warmup 10 \
  --modes native,vgpu --md-out $OUT/vgg_auto.md > $OUT/vgg_auto.log 2>&1 || { tail -20 $OUT/vgg_auto.log; exit 8; }
grep vgg16 $OUT/vgg_off.md $OUT/vgg_auto.md
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o vgg -- python3 benchmarks/aibench_suite.py \
  --cases vgg16-inf --steps 20 --warmup 10 --modes vgpu > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 10; }
python3 tools/prof_summary.py "$OUT/prof/**/*results.db" --after-last naive_conv --top 20 -o $OUT/prof_ss.md \
  --title "VGG-16 inference b=20 bf16 in a vGPU (r1v)" > /dev/null || true
