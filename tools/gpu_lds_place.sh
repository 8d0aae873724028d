#!/bin/bash
# Table-only LDS placement: parity tests, then the config-4 budget sweep and a config-2 check.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/lds_place
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_http_gpu.py tests/test_mixed_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.out 2>&1
rc=$?; echo "pytest rc=$rc"; tail -1 $OUT/pytest.out; [ $rc -eq 0 ] || exit $rc
for b in 0 65536 81920 98304; do
  timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --lds-budget $b > $OUT/b$b.json 2> $OUT/b$b.err || exit $?
  python -c "import json; d=json.load(open('$OUT/b$b.json')); print('cfg4', $b, round(d['ms_per_step'],3), d['counters_ok'])"
done
timeout -k 10 300 python -u bench.py --steps 5 --warmup 2 --no-cpu-baseline > $OUT/cfg2.json 2> $OUT/cfg2.err || exit $?
python -c "import json; d=json.load(open('$OUT/cfg2.json')); print('cfg2', round(d['ms_per_step'],3), d['counters_ok'])"
