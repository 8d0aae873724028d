#!/bin/bash
# A/B session: parity tests of the in-tree library (TESTS, default the HTTP
# GPU tests), then kernel time of the in-tree library and of every
# variants/*.so on the given configs (tools/build_variant.sh builds them).
#   TESTS="tests/test_http_gpu.py" CFGS="2 5" bash tools/gpu_ab.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-ab}
OUT=gpurun_out/$TAG
mkdir -p $OUT
TESTS=${TESTS:-"tests/test_http_gpu.py tests/test_policy_gpu.py"}
if [ "$TESTS" != "none" ]; then
  timeout -k 10 600 python -u -m pytest $TESTS -x -q --timeout 150 --timeout-method thread > $OUT/pytest.log 2>&1
  rc=$?; echo "pytest rc=$rc"; tail -2 $OUT/pytest.log
  [ $rc -eq 0 ] || exit $rc
fi
for cfg in ${CFGS:-2}; do
  for L in cilium_amd/libl7match.so variants/*.so; do
    [ -f "$L" ] || continue
    n=$(basename $L .so)
    L7M_LIB=$L timeout -k 10 300 python -u bench.py --config $cfg --steps ${STEPS:-20} --warmup 3 --no-cpu-baseline \
      --no-e2e --no-batcher > $OUT/bench_${n}_cfg$cfg.json 2> $OUT/bench_${n}_cfg$cfg.err
    rc=$?
    [ $rc -eq 0 ] || { echo "$n cfg$cfg rc=$rc"; tail -3 $OUT/bench_${n}_cfg$cfg.err; exit $rc; }
    python3 -c "import json; d=json.load(open('$OUT/bench_${n}_cfg$cfg.json')); r=d['roofline']; print('$n', 'cfg$cfg', round(r['kernel_ms'], 3), 'ms', round(r['frac'], 4), d.get('counters_ok'))"
  done
done
