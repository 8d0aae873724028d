#!/bin/bash
# Config 4 (mixed HTTP+Kafka): parity test, bench line, rocprof kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r01_mixed}
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_mixed_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.out 2>&1
rc=$?; echo "pytest rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 python -u bench.py --config 4 > $OUT/bench.out 2> $OUT/bench.err
rc=$?; echo "bench rc=$rc"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 420 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof -o run --output-format csv -- \
  python3 -u bench.py --config 4 --steps 20 --warmup 2 --no-cpu-baseline > $OUT/prof.out 2> $OUT/prof.err
rc=$?; echo "rocprof rc=$rc"; exit $rc
