#!/bin/bash
# Round-6 session G, on one box, alternated: the batcher (config 2, 8 eager
# callers, four flushers) with the default build, variants/spec
# (L7M_SPEC_TILE=1: a small batch's bytes requested before its offsets) and
# variants/spec2 (the same, and the deciding wave signals completion without
# the per-wave counter); then config 2's bulk launch, default vs spec2, to
# show the switch costs the 64 M-request kernel nothing.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6g}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
B="cilium_amd/batcher_bench 2 1000000 3 1 8"
for rep in 1 2 3; do
  step base_$rep 60 $B || exit $?
  LD_LIBRARY_PATH=$PWD/variants/spec step spec_$rep 60 $B || exit $?
  LD_LIBRARY_PATH=$PWD/variants/spec2 step spec2_$rep 60 $B || exit $?
done
A="--steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --parity-sample 50000"
for rep in 1 2; do
  step bulk_base_$rep 300 python3 -u bench.py $A || exit $?
  L7M_LIB=variants/spec2.so step bulk_spec2_$rep 300 python3 -u bench.py $A || exit $?
done
