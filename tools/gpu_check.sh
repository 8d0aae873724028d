#!/bin/bash
# One GPU session: parity tests, bench, rocprof kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout ends the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out
mkdir -p $OUT
TAG=${1:-r01}
BENCH_ARGS=${BENCH_ARGS:-}
stop_if_fatal() {  # $1 = rc, $2 = step
  case $1 in
    0|1) return 0 ;;
    *) echo "FATAL: $2 exited $1; stopping" | tee -a $OUT/steps.log; exit $1 ;;
  esac
}
echo "== pytest -m gpu" | tee -a $OUT/steps.log
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 150 --timeout-method thread > $OUT/pytest_gpu_$TAG.log 2>&1
rc=$?; echo "pytest rc=$rc" | tee -a $OUT/steps.log; stop_if_fatal $rc pytest
echo "== bench" | tee -a $OUT/steps.log
timeout -k 10 420 python -u bench.py $BENCH_ARGS > $OUT/bench_$TAG.json 2> $OUT/bench_$TAG.err
rc=$?; echo "bench rc=$rc" | tee -a $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
echo "== rocprofv3 kernel trace" | tee -a $OUT/steps.log
export TMPDIR=/tmp
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_$TAG -o run --output-format csv -- \
  python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline $BENCH_ARGS > $OUT/prof_bench_$TAG.log 2>&1
rc=$?; echo "rocprof rc=$rc" | tee -a $OUT/steps.log
exit $rc
