#!/bin/bash
# Round-6 session J, one box: flushers x launches in flight per flusher
# (L7M_IN_FLIGHT, L7M_PIPE), config 2 / 8 eager callers, four alternated
# rounds of the default (4, 1) against (1, 4) and (2, 3); then the same at
# 16 callers once each.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6j}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
for rep in 1 2 3 4; do
  for fp in 4_1 1_4 2_3; do
    f=${fp%_*}; p=${fp#*_}
    L7M_IN_FLIGHT=$f L7M_PIPE=$p step b_f${f}_p${p}_$rep 60 cilium_amd/batcher_bench 2 1000000 3 1 8 || exit $?
  done
done
for fp in 4_1 1_4 2_3; do
  f=${fp%_*}; p=${fp#*_}
  L7M_IN_FLIGHT=$f L7M_PIPE=$p step c16_f${f}_p${p} 60 cilium_amd/batcher_bench 2 1000000 3 1 16 || exit $?
done
