#!/bin/bash
# Round 2q: the whole GPU test suite (as the driver runs it at round end), then smoke().
out=gpurun_out/r2q; mkdir -p $out
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v --timeout 200 --timeout-method thread > $out/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc" >> $out/steps.txt; [ $rc -ne 0 ] && exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $out/smoke.log 2>&1
echo "smoke rc=$?" >> $out/steps.txt
