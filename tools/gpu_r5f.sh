#!/bin/bash
# Round-5 session F: RE2 alit placement A/B + timeline.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5f; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step re2_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_re2_gpu.py || exit $?
step re2_lds 300 python -u bench.py --dialect re2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e || exit $?
L7M_LIB=variants/prof.so step prof_re2 300 python -u bench.py --dialect re2 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity --requests 16000000 || exit $?
