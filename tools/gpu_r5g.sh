#!/bin/bash
# Round-5 session G: RE2 alit ablations (diagnostic variants, verdicts invalid).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5g; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
for v in skip onlyload_skip nocand_skip; do
  L7M_LIB=variants/$v.so step re2_$v 300 python -u bench.py --dialect re2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e --no-parity || exit $?
done
