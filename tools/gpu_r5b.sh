#!/bin/bash
# Round-5 session B: slow pass rework (work queue, LDS record slots).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5b; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step slow_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_regex_ext_gpu.py tests/test_abi_gpu.py tests/test_re2_gpu.py || exit $?
step bench_ext 400 python -u bench.py --extended --steps 5 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
step bench_re2 400 python -u bench.py --dialect re2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
