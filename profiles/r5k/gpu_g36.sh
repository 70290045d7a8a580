# Round-5 GPU study (profiles/r5k, part 5): 4 and 8 LSTM pods taking turns in pairs over the
# node board (VGPU_GPU_CONCURRENCY=2, 20 ms slices) vs all at once (default).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --case lstm-inf --tenants 4,8 --policy default --seconds 5 \
  --pod-env VGPU_GPU_CONCURRENCY=2 --json-out $out/lstm_conc2.json --md-out $out/lstm_conc2.md > $out/lstm_conc2.log 2>&1
rc=$?
cat $out/lstm_conc2.md
exit $rc
