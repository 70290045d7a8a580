set -o pipefail
# r1z: is the spatial-mode loss at 4+ tenants dispatcher-level? Interference of CU-masked
# tenants for grids that fit the slice at once (spin) vs grids dispatched over many rounds
# (spin-lds: 64 KiB LDS per workgroup), 4 and 8 tenants.
OUT=gpurun_out/r1z; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
for n in 4 8; do
  timeout -k 10 600 python benchmarks/spatial_interference.py --tenants $n --kinds spin,spin-lds \
    --md-out $OUT/interference_$n.md > $OUT/interference_$n.log 2>&1 || { tail -20 $OUT/interference_$n.log; exit 2; }
  cat $OUT/interference_$n.md
done
