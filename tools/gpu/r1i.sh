set -o pipefail
OUT=gpurun_out/r1i; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 900 python benchmarks/vgpu_scaling.py --policy shared,spatial,vdm --tenants 1,2,4,8,16 --json-out $OUT/scaling.json \
  --md-out $OUT/scaling.md > $OUT/scaling.log 2>&1; rc=$?; tail -18 $OUT/scaling.log; [ $rc -eq 0 ] || exit $rc
