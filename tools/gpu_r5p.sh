#!/bin/bash
# Round-5 session P: the default bench line of the final build (traffic from
# profiles/r05/traffic_cfg2.json, matched by the kernel hash).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5p; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python3 -u bench.py > $OUT/bench_default.out 2> $OUT/bench_default.err
echo "bench rc=$?" | tee -a $OUT/steps.log
