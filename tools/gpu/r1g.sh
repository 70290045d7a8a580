set -o pipefail
OUT=gpurun_out/r1g; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
timeout -k 10 900 python -m pytest tests -m gpu -q -rs -x -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -6 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python benchmarks/op_bench.py --md-out $OUT/op_bench.md > $OUT/op_bench.log 2>&1; rc=$?; tail -9 $OUT/op_bench.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python bench.py --steps 30 --warmup 10 --json-out $OUT/bench.json > $OUT/bench.log 2>&1; rc=$?; tail -1 $OUT/bench.log | cut -c1-300; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o bench -- python3 bench.py --steps 10 --warmup 10 --modes vgpu > $OUT/prof.log 2>&1; rc=$?; tail -1 $OUT/prof.log | cut -c1-200; [ $rc -eq 0 ] || exit $rc
