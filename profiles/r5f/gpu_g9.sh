# Round-5 GPU study (profiles/r5f): the suite's noisy cases re-measured - one case, native vs
# the quota-only vGPU, 8 ABBA repeats of a 10 s timed window each.
#   bash tools/gpu_g9.sh <case>
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5f
mkdir -p $out
c=$1
timeout -k 10 1050 python -u benchmarks/aibench_suite.py --cases $c --modes native,vgpu --repeats 8 --window 10 \
  --vdm 0 ${PIN:+--pin $PIN} --json-out $out/$c$TAG.json --md-out $out/$c$TAG.md > $out/$c$TAG.log 2>&1
rc=$?
echo "suite_rc=$rc" >> $out/$c$TAG.log
tail -6 $out/$c$TAG.log
exit $rc
