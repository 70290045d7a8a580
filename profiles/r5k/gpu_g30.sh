# Round-5 GPU study (profiles/r5k): packing launch-bound pods - 1/2/4/8 pods of a split-N
# plugin running LSTM inference (default policy and quota-only sharing), with the product's
# --numa-spread and with it turned off in the pods (VGPU_CPU_SPREAD=0); ResNet-152 b=10 with
# the spread.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5k
mkdir -p $out
S="timeout -k 10 400 python -u benchmarks/vgpu_scaling.py --tenants 1,2,4,8 --policy default,shared --seconds 5"
$S --case lstm-inf --json-out $out/lstm_spread.json --md-out $out/lstm_spread.md > $out/lstm_spread.log 2>&1 &&
cat $out/lstm_spread.md &&
$S --case lstm-inf --pod-env VGPU_CPU_SPREAD=0 --json-out $out/lstm_nospread.json --md-out $out/lstm_nospread.md > $out/lstm_nospread.log 2>&1 &&
cat $out/lstm_nospread.md &&
$S --case resnet152-inf --json-out $out/r152_spread.json --md-out $out/r152_spread.md > $out/r152_spread.log 2>&1 &&
cat $out/r152_spread.md
