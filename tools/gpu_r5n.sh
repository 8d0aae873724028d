#!/bin/bash
# Round-5 session N: RE2-dialect counters -- FETCH_SIZE / WRITE_SIZE of the
# 64 M-request launch (traffic) and the SQ passes (16 M requests).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5n; mkdir -p $OUT; export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_$ctr -o run --output-format csv -- \
    python3 -u bench.py --dialect re2 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher --no-parity > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc" | tee -a $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE 2 $OUT/traffic_cfg2_re2.json
echo "traffic rc=$?" | tee -a $OUT/steps.log
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--dialect re2 --no-parity" bash tools/gpu_pmc.sh sq_re2_r5n || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_sq_re2_r5n > gpurun_out/pmc_sq_re2_r5n/summary.txt
echo "summary rc=$?" | tee -a $OUT/steps.log
