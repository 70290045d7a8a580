#!/bin/bash
# Round-4 GPU check: the product's GPU tests (-x, as the driver runs them) at HEAD - SVM spill
# promotion and the lone-pod limiter bar included - then the lone-pod window arms (r4c lone).
out=${1:-gpurun_out/r4f}
mkdir -p "$out"
timeout -k 10 900 python -u -m pytest -x -v -rfE --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
bash profiles/r4c/r4_c.sh "$out" lone
