#!/bin/bash
# PMC passes of the Kafka kernel: full evaluation and the decode-only ablation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
P=${PASSES:-tools/pmc_passes2.txt}
BENCH_ARGS="--config 3" PASSES=$P REQS=16000000 bash tools/gpu_pmc.sh kafka_full || exit $?
BENCH_ARGS="--config 3 --diag walk" PASSES=$P REQS=16000000 bash tools/gpu_pmc.sh kafka_walk
