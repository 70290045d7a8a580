#!/bin/bash
# Round-4 final check (profiles/r4p): the product's GPU tests exactly as the driver runs them,
# then smoke(), at HEAD.
out=${1:-gpurun_out/r4p}
mkdir -p "$out"
timeout -k 10 1000 python -u -m pytest -x -v -rfEP --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
echo "smoke_rc=$?" >> "$out/smoke.log"
