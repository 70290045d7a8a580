#!/bin/bash
# Round-4 GPU check: the spill tests (SVM promotion, pinned backing) at HEAD.
out=${1:-gpurun_out/r4s}
mkdir -p "$out"
timeout -k 10 600 python -u -m pytest -x -v -rfEP --timeout 300 --timeout-method thread -m gpu \
  tests/test_gpu_limits.py -k "spill" -p no:cacheprovider > "$out/pytest.log" 2>&1
echo "pytest_rc=$?" >> "$out/pytest.log"
