set -o pipefail
# r1az: LSTM forward on buffer descriptors, backward back on global pointers (r1ay regression).
OUT=gpurun_out/r1az; mkdir -p $OUT; export TMPDIR=/tmp
make -C native -j16 > $OUT/build.log 2>&1 || exit 1
echo "pytest lstm"
timeout -k 10 300 python -u -m pytest tests/test_fused_ops.py -m gpu -k lstm -v -rs -x -p no:cacheprovider --timeout 120 \
  --timeout-method thread > $OUT/pytest_lstm.log 2>&1 || { tail -40 $OUT/pytest_lstm.log; exit 2; }
tail -3 $OUT/pytest_lstm.log
echo "suite fused"
timeout -k 10 400 python benchmarks/aibench_suite.py --cases lstm-train,lstm-inf --steps 20 --warmup 5 --repeats 1 \
  --modes native,vgpu,native-graph,vgpu-graph --json-out $OUT/suite.json --md-out $OUT/suite.md > $OUT/suite.log 2>&1 \
  || { tail -20 $OUT/suite.log; exit 3; }
cat $OUT/suite.md
echo "rocprof"
cd /tmp && VGPU_BENCH_GRAPH=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/$OUT/prof -o lstm -- \
  python3 $GRAFT_REPO_ROOT/benchmarks/aibench_suite.py --cases lstm-train --steps 10 --warmup 3 --json-out /tmp/p.json \
  --in-process > $GRAFT_REPO_ROOT/$OUT/prof.log 2>&1 || { tail -20 $GRAFT_REPO_ROOT/$OUT/prof.log; exit 5; }
ls $GRAFT_REPO_ROOT/$OUT/prof
