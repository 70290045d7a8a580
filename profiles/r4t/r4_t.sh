#!/bin/bash
# Round-4 final check (profiles/r4t): every GPU test, smoke() and bench.py at HEAD, in the
# driver's order.
out=${1:-gpurun_out/r4t}
mkdir -p "$out"
timeout -k 10 720 python -u -m pytest -x -v -rfEP --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
rc=$?
echo "smoke_rc=$rc" >> "$out/smoke.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 330 python -u bench.py --json-out "$out/bench.json" > "$out/bench.log" 2>&1
echo "bench_rc=$?" >> "$out/bench.log"
