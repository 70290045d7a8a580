# Round-5 GPU study (profiles/r5d): do two launch-bound processes' kernels overlap on one
# MI355X? 1 and 2 stock tenants (no shim, no CU mask) of LSTM inference and ResNet-152 b=10
# inference, without the profiler (aggregate throughput) and with a rocprofv3 kernel trace of
# every tenant, then the overlap / gap analysis of the traces.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
O=gpurun_out/r5d
mkdir -p $O
for c in lstm-inf resnet152-inf; do
  for n in 1 2; do
    timeout -k 10 240 python3 -u tools/probe/cotenancy.py --case $c --procs $n --seconds 4 > $O/plain_${c}_$n.json 2> $O/plain_${c}_$n.err || exit $?
    timeout -k 10 300 python3 -u tools/probe/cotenancy.py --case $c --procs $n --seconds 4 --trace /tmp/r5d_${c}_$n > $O/traced_${c}_$n.json 2> $O/traced_${c}_$n.err || exit $?
    python3 tools/probe/cotenancy.py --analyze /tmp/r5d_${c}_$n > $O/overlap_${c}_$n.json || exit $?
    tail -1 $O/plain_${c}_$n.json; cat $O/overlap_${c}_$n.json
  done
done
