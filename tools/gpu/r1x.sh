set -o pipefail
# r1x: concurrent-vGPU scaling curve on one MI355X with the MFMA conv kernels.
OUT=gpurun_out/r1x; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 1100 python benchmarks/vgpu_scaling.py --policy shared,spatial --tenants 1,2,4,8 --json-out $OUT/scaling.json \
  --md-out $OUT/scaling.md > $OUT/scaling.log 2>&1 || { tail -20 $OUT/scaling.log; exit 2; }
cat $OUT/scaling.md
