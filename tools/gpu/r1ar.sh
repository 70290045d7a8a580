set -o pipefail
# r1ar: headline step with each epilogue cache-policy build (ABAB order).
OUT=gpurun_out/r1ar; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for v in "" _both _ynt; do
    VGPU_OPS_LIB=libvgpu_ops$v.so timeout -k 10 600 python bench.py --steps 40 --warmup 10 --json-out $OUT/bench$v.$rep.json > $OUT/bench$v.$rep.log 2>&1 || { tail -20 $OUT/bench$v.$rep.log; exit 9; }
    echo "lib$v rep$rep $(python3 -c "import json;d=json.load(open('$OUT/bench$v.$rep.json'));print(d['value'], d['ms_per_step'])")"
  done
done
