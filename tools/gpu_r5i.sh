#!/bin/bash
# Round-5 session I: the whole GPU suite, then the RE2 line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5i; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step gpu_suite 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
step re2_bench 300 python -u bench.py --dialect re2 --steps 10 --warmup 2 --no-e2e || exit $?
