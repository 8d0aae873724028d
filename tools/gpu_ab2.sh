#!/bin/bash
# A/B session with variant parity: parity tests of the in-tree library
# (TESTS), then of each variant named in VTESTS ("name:testfile[,testfile]"
# items), then kernel time of the in-tree library and of every variants/*.so
# on CFGS.  Every GPU step has its own time limit; the first failure ends it.
#   TESTS="tests/test_kafka_gpu.py" VTESTS="kdma:tests/test_kafka_gpu.py" CFGS="3" bash tools/gpu_ab2.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
if [ -n "${TESTS:-}" ]; then
  timeout -k 10 900 python -u -m pytest $TESTS -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for item in ${VTESTS:-}; do
  n=${item%%:*}; files=${item#*:}
  L7M_LIB=variants/$n.so timeout -k 10 600 python -u -m pytest ${files//,/ } -x -q --timeout 200 --timeout-method thread \
    > $OUT/pytest_$n.log 2>&1
  rc=$?; echo "pytest[$n] rc=$rc"; tail -1 $OUT/pytest_$n.log
  [ $rc -eq 0 ] || exit $rc
done
for cfg in ${CFGS:-2}; do
  for L in cilium_amd/libl7match.so variants/*.so; do
    [ -f "$L" ] || continue
    n=$(basename $L .so)
    L7M_LIB=$L timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-e2e --no-batcher > $OUT/bench_${n}_cfg$cfg.out 2> $OUT/bench_${n}_cfg$cfg.err
    rc=$?
    [ $rc -eq 0 ] || { echo "$n cfg$cfg rc=$rc"; tail -3 $OUT/bench_${n}_cfg$cfg.err; exit $rc; }
    grep -h "L7M_QT\|L7M_PROF" $OUT/bench_${n}_cfg$cfg.out | head -4
    tail -1 $OUT/bench_${n}_cfg$cfg.out | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); r=d['roofline']; print('$n', 'cfg$cfg', round(r['kernel_ms'], 3), 'ms', round(r['frac'], 4), d.get('counters_ok'))"
  done
done
