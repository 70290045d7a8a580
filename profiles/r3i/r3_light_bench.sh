#!/bin/bash
# Round-3: the new light-tenant and hook-overhead GPU tests, then bench.py with the
# sweep extended to 12 and 16 pods (timings per sweep point in bench.log).
out=${1:-gpurun_out/r3i}
mkdir -p "$out"
timeout -k 10 420 python -u -m pytest -v -s --timeout 400 --timeout-method thread -m gpu \
  "tests/test_gpu_limits.py::test_temporal_four_light_tenants" tests/test_gpu_overhead.py \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 720 python -u bench.py --sweep-tenants 1,2,4,8,12,16 --json-out "$out/bench.json" > "$out/bench.log" 2>&1
