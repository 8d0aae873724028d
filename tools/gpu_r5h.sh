#!/bin/bash
# Round-5 session H: RE2 literal-anchored records (one read per candidate): parity + bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5h; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step re2_tests 400 python -u -m pytest tests/test_re2_gpu.py -x -v --timeout 120 --timeout-method thread || exit $?
step re2_bench 300 python -u bench.py --dialect re2 --steps 5 --warmup 1 --no-e2e || exit $?
