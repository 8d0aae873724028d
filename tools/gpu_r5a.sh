#!/bin/bash
# Round-5 session A: slow-pass tiers, device sets, resident batch test, then
# the full GPU suite and three bench lines.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5a; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step new_tests 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_re2_gpu.py tests/test_regex_ext_gpu.py tests/test_multi_gpu.py "tests/test_kafka_gpu.py::test_batcher_resident_recycled_batch_new_bytes_same_offsets" || exit $?
step all_tests 1100 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
step bench_ext 400 python -u bench.py --extended --steps 5 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
step bench_sp 400 python -u bench.py --single-process --devices 0,0 --requests 16000000 --steps 5 --warmup 1 || exit $?
step bench_re2 400 python -u bench.py --dialect re2 --steps 5 --warmup 1 --no-cpu-baseline --no-e2e || exit $?
step bench_default 400 python -u bench.py --no-cpu-baseline --no-batcher --no-e2e --steps 10 || exit $?
