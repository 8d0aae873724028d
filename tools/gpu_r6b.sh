#!/bin/bash
# Round-6 session B: A/B of the hit-counter slices (variants/slice.so:
# per-workgroup global counter slices, 8448-byte record stage) against the
# default build on config 2, alternated on one box; the default build's
# L7M_PROF wave timeline (variants/prof.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6b}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
A="--steps 20 --warmup 3 --no-cpu-baseline --no-e2e --no-batcher"
for i in 1 2; do
  step base_$i 300 python3 -u bench.py $A --parity-sample 50000 || exit $?
  L7M_LIB=variants/slice.so step slice_$i 300 python3 -u bench.py $A --parity-sample 50000 || exit $?
done
L7M_LIB=variants/prof.so step prof 300 python3 -u bench.py --requests 16000000 --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
