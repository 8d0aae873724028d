#!/bin/bash
# Parity tests, then bench variants (one process each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-sweep}
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 gpurun_out/pytest_$TAG.log; [ $rc -le 1 ] || exit $rc
shift
for v in "$@"; do
  timeout -k 10 200 python -u bench.py --no-cpu-baseline --steps 5 $v > gpurun_out/sw.json 2> gpurun_out/sw.err
  rc=$?; echo "[$v] rc=$rc $(tail -1 gpurun_out/sw.err)"; [ $rc -eq 0 ] || exit $rc
done
