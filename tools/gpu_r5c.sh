#!/bin/bash
# Round-5 session C: RE2 timeline (L7M_PROF variant), RE2 + default bench.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5c; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step bench_re2 400 python -u bench.py --dialect re2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-parity || exit $?
L7M_LIB=variants/prof.so step prof_re2 400 python -u bench.py --dialect re2 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity --requests 16000000 || exit $?
L7M_LIB=variants/prof.so step prof_default 400 python -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-parity --no-batcher --requests 16000000 || exit $?
step batcher 300 ./cilium_amd/batcher_bench 2 1000000 3 0 8 16 || exit $?
step batcher_eager 300 ./cilium_amd/batcher_bench 2 1000000 3 1 8 16 || exit $?
step bench_default 400 python -u bench.py --steps 10 --no-cpu-baseline --no-batcher --no-e2e || exit $?
