#!/bin/bash
# Round-5 session M (final build): config 2's FETCH_SIZE / WRITE_SIZE passes
# -> traffic per launch, the graft smoke test, the GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5m; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr" >> $OUT/steps.log
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_$ctr -o run --output-format csv -- \
    python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher --no-parity > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc" | tee -a $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE 2 $OUT/traffic_cfg2.json
echo "traffic rc=$?" | tee -a $OUT/steps.log
step smoke 300 python3 -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
step gpu_suite 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
