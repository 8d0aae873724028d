#!/bin/bash
# SQ counter passes (wave-cycle breakdown, LDS bank conflicts, VALU activity)
# of the HTTP (config 2) and Kafka (config 3) kernels: one rocprofv3 per pass.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r02}
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--config 2" bash tools/gpu_pmc.sh sq_http_$TAG || exit $?
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--config 3" bash tools/gpu_pmc.sh sq_kafka_$TAG || exit $?
python3 tools/pmc_summary.py gpurun_out/pmc_sq_http_$TAG > gpurun_out/pmc_sq_http_$TAG/summary.txt
python3 tools/pmc_summary.py gpurun_out/pmc_sq_kafka_$TAG > gpurun_out/pmc_sq_kafka_$TAG/summary.txt
