set -o pipefail
# r1at: prologue conv1 on LDS-DMA staging (BN+ReLU on the A fragments), packed bf16 stores.
OUT=gpurun_out/r1at; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_fused_ops.py -m gpu -x -q --timeout 120 --timeout-method thread \
  -p no:cacheprovider > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 6; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python benchmarks/conv_bench.py --md-out $OUT/conv.md > $OUT/conv.log 2>&1 || { tail -20 $OUT/conv.log; exit 7; }
python3 tools/conv_compare.py profiles/r1aq/conv.md $OUT/conv.md
timeout -k 10 300 python benchmarks/kernel_pmc.py --iters 20 > $OUT/pmc_smoke.log 2>&1 || { tail -5 $OUT/pmc_smoke.log; exit 8; }
for rep in 1 2; do
  for m in auto on; do
    VGPU_PROLOGUE=$m timeout -k 10 600 python bench.py --steps 40 --warmup 10 --json-out $OUT/bench_$m.$rep.json > $OUT/bench_$m.$rep.log 2>&1 || { tail -20 $OUT/bench_$m.$rep.log; exit 9; }
    echo "prologue=$m rep$rep $(python3 -c "import json;d=json.load(open('$OUT/bench_$m.$rep.json'));print(d['value'], d['ms_per_step'])")"
  done
done
