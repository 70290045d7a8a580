# Round-5 GPU run (profiles/r5i): the suite's VDM column for all ten cases - two concurrent
# pods of the reference's split-2 DaemonSet config, placed by the product (--numa-spread) -
# with one native / vGPU repeat for the table.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5i
mkdir -p $out
timeout -k 10 1100 python -u benchmarks/aibench_suite.py --cases all --modes native,vgpu --repeats 1 --steps 10 \
  --vdm 1 --vdm-seconds 5 --json-out $out/suite_vdm.json --md-out $out/suite_vdm.md > $out/suite_vdm.log 2>&1
rc=$?
echo "suite_rc=$rc" >> $out/suite_vdm.log
cat $out/suite_vdm.md
exit $rc
