# Round-5 GPU study (profiles/r5k, part 4): 4 and 8 LSTM pods on disjoint CU slices
# (--cu-mode spatial) vs the default policy (GPU-time limiter at 4 and 8).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --case lstm-inf --tenants 1,4,8 --policy spatial,default --seconds 5 \
  --json-out $out/lstm_spatial.json --md-out $out/lstm_spatial.md > $out/lstm_spatial.log 2>&1
rc=$?
cat $out/lstm_spatial.md
exit $rc
