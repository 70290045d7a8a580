set -o pipefail
# r1ac: persistent (capped) conv grids inside CU-masked vGPUs: numerics, bench, spatial scaling.
OUT=gpurun_out/r1ac; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1 || { tail -20 $OUT/bench.log; exit 9; }
cut -c1-160 $OUT/bench.json
timeout -k 10 1000 python benchmarks/vgpu_scaling.py --policy spatial --tenants 4,8 --json-out $OUT/scaling.json \
  --md-out $OUT/scaling.md > $OUT/scaling.log 2>&1 || { tail -20 $OUT/scaling.log; exit 2; }
cat $OUT/scaling.md
