#!/bin/bash
# A subset of the GPU tests (paths as arguments), each run under its own time limit, output
# under gpurun_out/<tag>/. Usage: bash tools/gpu/tests_subset.sh <tag> <test paths...>
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest "$@" -m gpu -x -v -s -rs -p no:cacheprovider --timeout 600 > $OUT/pytest.log 2>&1
rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; exit $rc
