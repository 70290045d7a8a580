set -o pipefail
OUT=gpurun_out/r1f; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 300 python tools/gpu/smi_diag.py > $OUT/smi_diag.log 2>&1; rc=$?; cat $OUT/smi_diag.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python benchmarks/vgpu_scaling.py --policy spatial-q1,shared --tenants 2,4,8 --md-out $OUT/scaling_q1.md > $OUT/scaling_q1.log 2>&1; rc=$?; tail -9 $OUT/scaling_q1.log; [ $rc -eq 0 ] || exit $rc
for t in 0 1; do
  timeout -k 10 600 python bench.py --steps 30 --warmup 10 --tune $t --json-out $OUT/bench_tune$t.json > $OUT/bench_tune$t.log 2>&1 || exit 1
  tail -1 $OUT/bench_tune$t.log | cut -c1-200
done
