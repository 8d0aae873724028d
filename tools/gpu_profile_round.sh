#!/bin/bash
# Round profile set (run on the GPU box): rocprofv3 kernel-trace summaries of
# configs 2-5, FETCH_SIZE / WRITE_SIZE passes (HBM traffic per launch) of
# configs 2, 3 and 5, SQ passes of configs 2 and 3, and the default bench line.
#   tools/gpu_profile_round.sh TAG      -> gpurun_out/TAG/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-prof}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in 2 3 4 5; do
  timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/cfg$cfg -o run --output-format csv -- \
    python3 -u bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher > $OUT/cfg$cfg.json 2> $OUT/cfg$cfg.err
  rc=$?; echo "trace cfg$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
for cfg in 2 3 5; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_${cfg}_$ctr -o run --output-format csv -- \
      python3 -u bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher > $OUT/pmc_${cfg}_$ctr.log 2>&1
    rc=$?; echo "pmc cfg$cfg $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
done
bash tools/gpu_sq.sh $TAG || exit $?
timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err
echo "bench rc=$?"
