set -o pipefail
OUT=gpurun_out/r1l; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -rs -x -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -4 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/temporal_accuracy.py --md-out $OUT/temporal.md > $OUT/temporal.log 2>&1; rc=$?; tail -6 $OUT/temporal.log; [ $rc -eq 0 ] || exit $rc
