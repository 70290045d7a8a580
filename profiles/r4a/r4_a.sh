#!/bin/bash
# Round-4 first GPU check (profiles/r4a):
#   1. light tenants study: native x1/x4, unlimited x4, limited 25 % x1/x4, and the limited
#      arms again with the shim of 59cfc76 (the build behind profiles/r3c) - A/B for the
#      round-3 drop of the four light tenants' aggregate;
#   2. the product's GPU tests (all of them, not stopping at the first failure);
#   3. smoke().
# Each GPU step has its own time limit; a crash/timeout ends the script.
out=${1:-gpurun_out/r4a}
mkdir -p "$out"
ab=4paradigm-k8s-device-plugin_amd/lib/ab/libvgpu_hip_59cfc76.so
timeout -k 10 600 python -u benchmarks/light_tenants.py --seconds 5 --repeats 2 --ab-shim "$ab" \
  --json-out "$out/light.json" --md-out "$out/light.md" > "$out/light.log" 2>&1
rc=$?
echo "light_rc=$rc" >> "$out/light.log"
case $rc in 0) ;; *) exit $rc ;; esac
timeout -k 10 1200 python -u -m pytest -v -rfE --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
echo "smoke_rc=$?" >> "$out/smoke.log"
