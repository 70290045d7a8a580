set -o pipefail
OUT=gpurun_out/r1h; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 1000 python benchmarks/aibench_suite.py --steps 20 --warmup 10 --repeats 2 --modes native,vgpu,vgpu-cu50 \
  --json-out $OUT/suite.json --md-out $OUT/suite.md > $OUT/suite.log 2>&1; rc=$?; tail -14 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/temporal_accuracy.py --md-out $OUT/temporal.md > $OUT/temporal.log 2>&1; rc=$?; tail -6 $OUT/temporal.log; [ $rc -eq 0 ] || exit $rc
