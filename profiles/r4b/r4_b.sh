#!/bin/bash
# Round-4 GPU check 2 (profiles/r4b): can ROCr back a GPU-visible VMM range with host memory
# (native/tests/vmem_probe.hip) or KFD's SVM ranges migrate between host and HBM without XNACK
# (native/tests/svm_probe.hip; status codes only before any kernel touches a range); hook cost at
# HEAD (C++ probe, with the gates made pass-throughs and the dlsym routing off as
# diagnostics); then the product's GPU tests exactly as the driver runs them (-x), then smoke().
out=${1:-gpurun_out/r4b}
mkdir -p "$out"
timeout -k 10 60 4paradigm-k8s-device-plugin_amd/lib/vmem_probe 64 > "$out/vmem.json" 2> "$out/vmem.err"
rc=$?
echo "vmem_rc=$rc" >> "$out/vmem.err"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 90 4paradigm-k8s-device-plugin_amd/lib/svm_probe 256 > "$out/svm.json" 2> "$out/svm.err"
rc=$?
echo "svm_rc=$rc" >> "$out/svm.err"
case $rc in 0|1) ;; *) exit $rc ;; esac
timeout -k 10 300 python -u benchmarks/hook_overhead.py --probe --repeats 3 --iters 10000 \
  --modes native,vgpu,vgpu-nogate,vgpu-nodlsym --json-out "$out/probe.json" --md-out "$out/probe.md" \
  > "$out/probe.log" 2>&1 || exit $?
timeout -k 10 900 python -u -m pytest -x -v -rfE --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 150 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
echo "smoke_rc=$?" >> "$out/smoke.log"
