set -o pipefail
# r1as: conv1 prologue only where conv1 is memory-bound (Cout <= 128) vs everywhere (ABAB).
OUT=gpurun_out/r1as; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider -k "resnet" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
for rep in 1 2; do
  for m in auto on; do
    VGPU_PROLOGUE=$m timeout -k 10 600 python bench.py --steps 40 --warmup 10 --json-out $OUT/bench_$m.$rep.json > $OUT/bench_$m.$rep.log 2>&1 || { tail -20 $OUT/bench_$m.$rep.log; exit 9; }
    echo "prologue=$m rep$rep $(python3 -c "import json;d=json.load(open('$OUT/bench_$m.$rep.json'));print(d['value'], d['ms_per_step'])")"
  done
done
