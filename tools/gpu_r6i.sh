#!/bin/bash
# Round-6 session I, one box: the batcher with several kernel-signalled
# launches in flight per flusher (L7M_PIPE, l7m_batch.cc Slot) -- the GPU
# batcher tests at pipe 1 and 2, then config 2 / 8 eager callers for
# (flushers, pipe) pairs, alternated.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6i}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
T="python3 -u -m pytest tests/test_abi_gpu.py tests/test_kafka_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -k batcher"
step tests_p1 300 $T || exit $?
L7M_PIPE=2 step tests_p2 300 $T || exit $?
B="cilium_amd/batcher_bench 2 1000000 3 1 8"
for rep in 1 2; do
  for fp in 4_1 2_2 3_2 2_3 1_4; do
    f=${fp%_*}; p=${fp#*_}
    L7M_IN_FLIGHT=$f L7M_PIPE=$p step b_f${f}_p${p}_$rep 60 $B || exit $?
  done
done
