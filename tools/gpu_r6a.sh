#!/bin/bash
# Round-6 session A: the GPU suite as the driver runs it (-x), then fresh SQ
# counters of the shipped ECMAScript kernel (config 2, 16 M requests) and the
# default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r6a}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step gpu_suite 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
step bench_default 600 python3 -u bench.py || exit $?
step bench_ext 400 python3 -u bench.py --extended --no-batcher --no-e2e || exit $?
step bench_re2 400 python3 -u bench.py --dialect re2 --no-batcher --no-e2e || exit $?
step trace_ext 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace_ext -o run --output-format csv -- \
  python3 -u bench.py --extended --steps 10 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--no-parity" bash tools/gpu_pmc.sh sq_http_$TAG > $OUT/pmc.log 2>&1
echo "pmc rc=$?" | tee -a $OUT/steps.log
python3 tools/pmc_summary.py gpurun_out/pmc_sq_http_$TAG > $OUT/sq_summary.txt 2>&1
echo "summary rc=$?" | tee -a $OUT/steps.log
