#!/bin/bash
# Config 4: LDS table budget sweep (HTTP part's 52 KiB path table in or out of LDS).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mixed_lds
mkdir -p $OUT
for b in 0 65536 81920 98304; do
  timeout -k 10 300 python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline --lds-budget $b > $OUT/b$b.json 2> $OUT/b$b.err || exit $?
  python -c "import json; d=json.load(open('$OUT/b$b.json')); print($b, round(d['ms_per_step'],3), d['counters_ok'])"
done
