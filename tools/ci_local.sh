#!/bin/bash
# The CI workflow's build-test job (.github/workflows/ci.yml) on this machine, minus the
# dependency installation step (no network; the same packages are preinstalled):
#   tools/ci_local.sh [LOG]
set -o pipefail
log=${1:-/dev/stdout}
cd "$(dirname "$0")/.."
{
  echo "# ci_local $(date -u +%FT%TZ) $(git rev-parse --short HEAD 2>/dev/null)"
  echo "## native build" && make -C native -j4 2>&1 | tail -3 &&
  echo "## image rehearsal" && python3 tools/image_rehearsal.py 2>&1 | tail -3 &&
  echo "## tests (no GPU)" && python3 -m pytest tests -q -m "not gpu" --timeout 600 -p no:cacheprovider 2>&1 | tail -3
  rc=$?
  echo "## exit $rc"
  exit $rc
} > "$log" 2>&1
