#!/bin/bash
# Round-end style GPU session: parity tests, default bench (HTTP config 2 with
# CPU baseline), Kafka bench (config 3), rocprof kernel-trace summaries, and
# the FETCH_SIZE / WRITE_SIZE passes for the HBM traffic of the bench kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r01}
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc"; return $rc
}
step pytest_gpu 420 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread
rc=$?; [ $rc -le 1 ] || exit $rc
step bench_http 420 python -u bench.py || exit 1
step bench_kafka 420 python -u bench.py --config 3 || exit 1
step prof_http 420 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_http -o run --output-format csv -- python3 -u bench.py --steps 20 --warmup 2 --no-cpu-baseline || exit 1
step prof_kafka 420 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_kafka -o run --output-format csv -- python3 -u bench.py --config 3 --steps 20 --warmup 2 --no-cpu-baseline || exit 1
for c in FETCH_SIZE WRITE_SIZE; do
  for cfg in 2 3; do
    step pmc_${c}_$cfg 180 rocprofv3 --pmc $c -d $PWD/$OUT/pmc_${c}_$cfg -o run --output-format csv -- python3 -u bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline || exit 1
  done
done
