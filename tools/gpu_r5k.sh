#!/bin/bash
# Round-5 session K: config 5 with dynamic chunk assignment (in-tree .so) vs the
# static per-wave shares (variants/static.so), alternated; config-5 GPU parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5k; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step adv_tests 600 python -u -m pytest tests/test_adversarial_gpu.py -x -v --timeout 300 --timeout-method thread || exit $?
for i in 1 2; do
  step cfg5_dyn_$i 300 python -u bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
  L7M_LIB=variants/static.so step cfg5_static_$i 300 python -u bench.py --config 5 --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
done
