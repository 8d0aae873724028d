#!/bin/bash
# SQ counter passes of the final round-6 device code (tools/pmc_sq.txt: wave
# cycles, waits, VALU / SALU / LDS instructions, LDS bank conflicts) for
# config 2 (ECMAScript), config 3 (Kafka) and config 2 in the RE2 dialect,
# 16 M requests each; one rocprofv3 process per pass (tools/gpu_pmc.sh).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r6h}
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--config 2" bash tools/gpu_pmc.sh sq_http_$TAG || exit $?
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--config 3" bash tools/gpu_pmc.sh sq_kafka_$TAG || exit $?
PASSES=tools/pmc_sq.txt REQS=16000000 BENCH_ARGS="--dialect re2" bash tools/gpu_pmc.sh sq_re2_$TAG || exit $?
for k in http kafka re2; do
  python3 tools/pmc_summary.py gpurun_out/pmc_sq_${k}_$TAG > gpurun_out/pmc_sq_${k}_$TAG/summary.txt || exit $?
done
