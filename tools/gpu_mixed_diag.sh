#!/bin/bash
# Config 4 HTTP-part diagnosis: default build, no counters, 8K LDS-counter build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/mixed_diag
mkdir -p $OUT
B="python -u bench.py --config 4 --steps 5 --warmup 2 --no-cpu-baseline"
timeout -k 10 300 $B > $OUT/default.json 2> $OUT/default.err || exit $?
timeout -k 10 300 $B --no-hits > $OUT/nohits.json 2> $OUT/nohits.err || exit $?
L7M_LIB=$PWD/cilium_amd/libl7match_c8k.so timeout -k 10 300 $B > $OUT/c8k.json 2> $OUT/c8k.err || exit $?
for f in default nohits c8k; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', round(d['ms_per_step'],3), d['counters_ok'])"; done
