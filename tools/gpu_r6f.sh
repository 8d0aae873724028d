#!/bin/bash
# Round-6 session F, on one box: the batcher (config 2, 8 eager callers) with
#  - flushers x HIP hardware queues per process (each flusher launches on its
#    own stream; with GPU_MAX_HW_QUEUES=4, HIP's default, more than four
#    streams share hardware queues), and
#  - variants/spec (L7M_SPEC_TILE=1: a small batch's bytes requested before
#    its offsets arrive) against the default build,
# alternated; config 3 at the defaults and with 8 queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6f}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
B="cilium_amd/batcher_bench 2 1000000 3 1 8"
for rep in 1 2; do
  for q in 4 8; do
    for f in 4 6; do
      GPU_MAX_HW_QUEUES=$q L7M_IN_FLIGHT=$f step base_q${q}_f${f}_$rep 60 $B || exit $?
      LD_LIBRARY_PATH=$PWD/variants/spec GPU_MAX_HW_QUEUES=$q L7M_IN_FLIGHT=$f step spec_q${q}_f${f}_$rep 60 $B || exit $?
    done
  done
  GPU_MAX_HW_QUEUES=8 L7M_IN_FLIGHT=8 step base_q8_f8_$rep 60 $B || exit $?
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q step kafka_q${q} 60 cilium_amd/batcher_bench 3 1000000 3 1 8 || exit $?
done
