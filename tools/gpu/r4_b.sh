#!/bin/bash
# Round-4 GPU check 2 (profiles/r4b): hook cost at HEAD (C++ probe and PyTorch, with the
# gates made pass-throughs and the dlsym routing off as diagnostics), then the product's
# GPU tests exactly as the driver runs them (-x), then smoke().
out=${1:-gpurun_out/r4b}
mkdir -p "$out"
timeout -k 10 300 python -u benchmarks/hook_overhead.py --probe --repeats 3 --iters 10000 \
  --modes native,vgpu,vgpu-nogate,vgpu-nodlsym --json-out "$out/probe.json" --md-out "$out/probe.md" \
  > "$out/probe.log" 2>&1 || exit $?
timeout -k 10 400 python -u benchmarks/hook_overhead.py --repeats 3 --iters 20000 \
  --modes native,vgpu,vgpu-nogate,vgpu-nodlsym --json-out "$out/torch.json" --md-out "$out/torch.md" \
  > "$out/torch.log" 2>&1 || exit $?
timeout -k 10 1100 python -u -m pytest -x -v -rfE --timeout 300 --timeout-method thread -m gpu tests/ \
  -p no:cacheprovider > "$out/pytest.log" 2>&1
rc=$?
echo "pytest_rc=$rc" >> "$out/pytest.log"
case $rc in 124|134|137|139) exit $rc ;; esac
timeout -k 10 200 python -u -c "import __graft_entry__ as g; g.smoke()" > "$out/smoke.log" 2>&1
echo "smoke_rc=$?" >> "$out/smoke.log"
