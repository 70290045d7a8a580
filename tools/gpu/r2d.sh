#!/bin/bash
# Round 2d: product GPU tests after the limiter / host-PID / accounting rework.
out=gpurun_out/r2d; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests/test_gpu_limits.py tests/test_gpu_shim.py tests/test_gpu_control.py tests/test_gpu_e2e.py -v -s --timeout 240 --timeout-method thread > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/steps.txt
