#!/bin/bash
# Round-5 session O: RE2 wave timeline of the final kernel (L7M_PROF build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r5o; mkdir -p $OUT; export TMPDIR=/tmp
L7M_LIB=variants/prof.so timeout -k 10 300 python -u bench.py --dialect re2 --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher --no-parity --requests 16000000 > $OUT/prof_re2.out 2> $OUT/prof_re2.err
echo "prof_re2 rc=$?" | tee -a $OUT/steps.log
