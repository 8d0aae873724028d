#!/bin/bash
# Round-5 session L: full-match fields split their short-prefix patterns off
# an inflated automaton (config 2 + extended rules): parity on the GPU, the
# extended line, the default line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5l; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step ext_tests 600 python -u -m pytest tests/test_regex_ext_gpu.py -x -v --timeout 300 --timeout-method thread || exit $?
step bench_ext 400 python3 -u bench.py --extended --no-batcher || exit $?
step trace_ext 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace_ext -o run --output-format csv -- \
    python3 -u bench.py --extended --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
step bench_default 400 python3 -u bench.py --no-batcher || exit $?
