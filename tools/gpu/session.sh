#!/bin/bash
# One gpurun session: build, GPU tests, smoke, bench, rocprof profile.
# Usage (from the repo root, on the box):  bash tools/gpu/session.sh <tag> [steps...]
# steps: build tests smoke bench prof (default: all). Every GPU step has its own time
# limit and the script stops at the first failure.
set -o pipefail
TAG=${1:-run}; shift
STEPS=${*:-"build tests smoke bench prof"}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
has() { [[ " $STEPS " == *" $1 "* ]]; }
step() { echo "== $1 $(date +%T)"; }
if has build; then
  step build
  make -C native -j16 > $OUT/build.log 2>&1 || { echo "build failed"; tail -20 $OUT/build.log; exit 1; }
fi
if has tests; then
  step tests
  timeout -k 10 1000 python -u -m pytest tests -m gpu -x -v -rs -p no:cacheprovider > $OUT/pytest_gpu.log 2>&1
  rc=$?; tail -15 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
fi
if has smoke; then
  step smoke
  timeout -k 10 600 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
fi
if has bench; then
  step bench
  timeout -k 10 900 python bench.py --steps 20 --warmup 5 --json-out $OUT/bench.json > $OUT/bench.log 2>&1
  rc=$?; tail -3 $OUT/bench.log; [ $rc -eq 0 ] || exit $rc
fi
if has suite; then
  step suite
  timeout -k 10 1000 python benchmarks/aibench_suite.py --steps 20 --warmup 10 --repeats ${SUITE_REPEATS:-2} --modes ${SUITE_MODES:-native,vgpu,vgpu-cu50} \
    --json-out $OUT/suite.json --md-out $OUT/suite.md > $OUT/suite.log 2>&1
  rc=$?; tail -16 $OUT/suite.log; [ $rc -eq 0 ] || exit $rc
fi
if has scaling; then
  step scaling
  timeout -k 10 900 python benchmarks/vgpu_scaling.py --policy ${SCALING_POLICY:-spatial,shared} --json-out $OUT/scaling.json --md-out $OUT/scaling.md \
    > $OUT/scaling.log 2>&1
  rc=$?; tail -14 $OUT/scaling.log; [ $rc -eq 0 ] || exit $rc
fi
if has hooks; then
  step hooks
  timeout -k 10 600 python benchmarks/hook_overhead.py --json-out $OUT/hooks.json --md-out $OUT/hooks.md \
    > $OUT/hooks.log 2>&1
  rc=$?; tail -8 $OUT/hooks.log; [ $rc -eq 0 ] || exit $rc
fi
if has oversub; then
  step oversub
  timeout -k 10 600 python benchmarks/oversubscribe.py --json-out $OUT/oversub.json > $OUT/oversub.log 2>&1
  rc=$?; tail -4 $OUT/oversub.log; [ $rc -eq 0 ] || exit $rc
fi
if has prof; then
  step prof
  # rocprofv3 --kernel-trace --marker-trace --stats of the headline tenant: native, quota-only
  # vGPU, 25 % temporal vGPU (tools/probe/prof_tenant.py: each mode a child under its own
  # rocprofv3, the program after --; summary.md + per-mode kernel stats)
  timeout -k 10 700 python -u tools/probe/prof_tenant.py --out $OUT/prof --steps 30 > $OUT/prof.log 2>&1
  rc=$?; head -12 $OUT/prof/summary.md 2>/dev/null; [ $rc -eq 0 ] || exit $rc
fi
echo "== done $(date +%T)"
