#!/bin/bash
# Round 2ab: SMI virtualisation after rocm_smi index remapping (amd-smi / rocm-smi tests).
out=gpurun_out/r2ab; mkdir -p $out
timeout -k 10 400 python -u -m pytest tests/test_gpu_e2e.py tests/test_gpu_shim.py -k "smi" -v -s --timeout 200 --timeout-method thread > $out/pytest.log 2>&1
echo "pytest rc=$?" >> $out/steps.txt
