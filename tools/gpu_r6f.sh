#!/bin/bash
# Round-6 session F: batcher flushers x HIP hardware queues per process, on
# one box (config 2, 8 eager callers; config 3 at the defaults and with 8
# queues).  Each flusher launches on its own stream; with GPU_MAX_HW_QUEUES=4
# (HIP's default) more than four streams share hardware queues.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-r6f}; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
for rep in 1 2; do
  for q in 4 8; do
    for f in 3 4 6 8; do
      GPU_MAX_HW_QUEUES=$q L7M_IN_FLIGHT=$f step b2_q${q}_f${f}_$rep 60 cilium_amd/batcher_bench 2 1000000 3 1 8 || exit $?
    done
  done
done
for q in 4 8; do
  GPU_MAX_HW_QUEUES=$q step b3_q${q} 60 cilium_amd/batcher_bench 3 1000000 3 1 8 || exit $?
done
