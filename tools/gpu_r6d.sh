#!/bin/bash
# Round-6 session D: RE2 literal-anchored scan prefilter A/B on one box --
# default build (2^14-bit prefilter), variants/bloom12.so (2^12 bits),
# variants/nobloom.so (round-5 scan: every position reads its bucket).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6d}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
A="--dialect re2 --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --parity-sample 50000"
for i in 1 2; do
  step b14_$i 300 python3 -u bench.py $A || exit $?
  L7M_LIB=variants/bloom12.so step b12_$i 300 python3 -u bench.py $A || exit $?
  L7M_LIB=variants/nobloom.so step b0_$i 300 python3 -u bench.py $A || exit $?
done
