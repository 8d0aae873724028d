#!/bin/bash
# SQ passes of config 2 for the default build and with an env knob set
# (A/B of a compiler option): tools/gpu_sq_ab.sh TAG VAR=value
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; KV=$2
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--config 2" bash tools/gpu_pmc.sh sqa_$TAG || exit $?
export "$KV"
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--config 2" bash tools/gpu_pmc.sh sqb_$TAG || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_sqa_$TAG > gpurun_out/pmc_sqa_$TAG/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc_sqb_$TAG > gpurun_out/pmc_sqb_$TAG/summary.txt
