#!/bin/bash
# Round-3 GPU check: the product's GPU tests (new gate / compiled-tenant / pinned-memory
# tests first), then smoke(). Each GPU step has its own time limit; output under $1.
out=${1:-gpurun_out/r3}
mkdir -p "$out"
timeout -k 10 1000 python -u -m pytest -v -rfE --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
echo "smoke_rc=$?" >> "$out/smoke.log"
