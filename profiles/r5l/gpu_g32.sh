# Round-5 GPU profile (profiles/r5l): rocprofv3 kernel + marker trace of the headline tenant
# at HEAD - natively, in a quota-only vGPU and in a 25 % temporal vGPU (shim roctx ranges on).
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
out=gpurun_out/r5l
mkdir -p $out
timeout -k 10 700 python -u tools/probe/prof_tenant.py --out $out/prof --steps 30 > $out/prof.log 2>&1
rc=$?
cat $out/prof/summary.md 2>/dev/null | head -60
exit $rc
