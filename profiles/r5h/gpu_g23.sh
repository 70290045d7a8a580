# Round-5 final check, part 2: smoke() and the driver's default bench at HEAD.
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/r5h
timeout -k 10 300 python -u -m pytest -v -s --timeout 280 --timeout-method thread -p no:cacheprovider -m gpu \
  "tests/test_gpu_limits.py::test_background_class_yields_to_a_busy_latency_class" > gpurun_out/r5h/bg_test.log 2>&1
rc=$?
grep -E "next_to_equal|PASSED|FAILED" gpurun_out/r5h/bg_test.log | cut -c1-600
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r5h/smoke.log 2>&1 || { tail -20 gpurun_out/r5h/smoke.log; exit 1; }
tail -2 gpurun_out/r5h/smoke.log
timeout -k 10 660 python -u bench.py --json-out gpurun_out/r5h/bench.json > gpurun_out/r5h/bench.log 2>&1
rc=$?
tail -1 gpurun_out/r5h/bench.log | cut -c1-600
python3 -c "
import json; d=json.load(open('gpurun_out/r5h/bench.json'))
print('max_vgpus_per_gpu', d.get('max_vgpus_per_gpu'))
for p in d.get('sweep', []):
    print(p.get('tenants'), p.get('aggregate_vs_one'), p.get('min_tenant_vs_entitlement'), p.get('cpus_busy'), p.get('skipped', ''))
"
exit $rc
