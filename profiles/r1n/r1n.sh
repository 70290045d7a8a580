set -o pipefail
# r1n: rocprof PMC evidence of CU confinement; BASELINE config 3 (two VGG-16 training
# tenants at 50 % CUs); MFMA 1x1 conv with fused epilogue: numerics, per-layer A/B, bench.
OUT=gpurun_out/r1n; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
PMC="SQ_WAVES SQ_BUSY_CU_CYCLES GRBM_GUI_ACTIVE SIMD_UTILIZATION"
for lim in 0 50 25; do
  echo "pmc cu_limit=$lim"
  VGPU_CONV1X1=off timeout -s KILL 240 rocprofv3 --pmc $PMC --kernel-trace --output-format csv \
    -d $OUT/pmc_cu$lim -o cu$lim -- python3 benchmarks/cu_occupancy.py --cu-limit $lim > $OUT/pmc_cu$lim.log 2>&1 \
    || { tail -20 $OUT/pmc_cu$lim.log; exit 3; }
done
python3 tools/pmc_summary.py "native=$OUT/pmc_cu0/**/*counter_collection.csv" \
  "vgpu-cu50=$OUT/pmc_cu50/**/*counter_collection.csv" "vgpu-cu25=$OUT/pmc_cu25/**/*counter_collection.csv" \
  --title "CU confinement by hardware counters (rocprofv3 --pmc), ResNet-V2-50 inference + spin" \
  -o $OUT/pmc_summary.md > /dev/null || exit 4
echo "config 3"
VGPU_CONV1X1=off timeout -k 10 900 python benchmarks/vgpu_scaling.py --case vgg16-train --tenants 1,2 \
  --policy spatial,shared --steps 30 --warmup 5 --json-out $OUT/config3.json --md-out $OUT/config3.md \
  > $OUT/config3.log 2>&1 || { tail -20 $OUT/config3.log; exit 5; }
echo "conv1x1 tests"
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -v --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "conv1x1" > $OUT/pytest_conv1x1.log 2>&1 || { tail -30 $OUT/pytest_conv1x1.log; exit 6; }
tail -2 $OUT/pytest_conv1x1.log
echo "conv1x1 bench"
timeout -k 10 600 python benchmarks/conv1x1_bench.py --md-out $OUT/conv1x1.md --json-out $OUT/conv1x1.json \
  > $OUT/conv1x1.log 2>&1 || { tail -20 $OUT/conv1x1.log; exit 7; }
tail -14 $OUT/conv1x1.log | cut -c1-200
echo "bench A/B"
VGPU_CONV1X1=off timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench_off.json \
  > $OUT/bench_off.log 2>&1 || { tail -20 $OUT/bench_off.log; exit 8; }
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench_auto.json \
  > $OUT/bench_auto.log 2>&1 || { tail -20 $OUT/bench_auto.log; exit 9; }
cut -c1-400 $OUT/bench_off.json $OUT/bench_auto.json
