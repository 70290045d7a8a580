set -o pipefail
OUT=gpurun_out/r1m; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 600 python benchmarks/spatial_interference.py --tenants 4 --md-out $OUT/interference.md > $OUT/interference.log 2>&1; rc=$?; tail -7 $OUT/interference.log; [ $rc -eq 0 ] || exit $rc
