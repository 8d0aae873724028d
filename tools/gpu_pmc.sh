#!/bin/bash
# PMC passes over a short bench run (one rocprofv3 process per pass).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/pmc_${1:-r01}
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--requests ${REQS:-8000000} --steps 2 --warmup 1 --no-cpu-baseline --no-e2e --no-batcher ${BENCH_ARGS:-}"
if [ "${LIST:-0}" = 1 ]; then
  timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1; echo "list rc=$?"
fi
i=0
while read -r pass; do
  [ -z "$pass" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $pass -d $PWD/$OUT/p$i -o run --output-format csv -- python3 -u bench.py $ARGS > $OUT/p$i.log 2>&1
  rc=$?; echo "pass $i ($pass) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done < ${PASSES:-tools/pmc_passes.txt}
