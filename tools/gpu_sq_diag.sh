#!/bin/bash
# SQ pass 1 (instruction mix) of config 2 for the full kernel and its copy-only
# and walk-only diagnostic instantiations: tools/gpu_sq_diag.sh TAG [cfg]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFG=${2:-2}
head -1 tools/pmc_sq.txt > /tmp/pass1.txt
for d in full copy walk; do
  extra=""; [ $d != full ] && extra="--diag $d"
  PASSES=/tmp/pass1.txt REQS=16000000 BENCH_ARGS="--config $CFG $extra" bash tools/gpu_pmc.sh sqd_${TAG}_$d || exit $?
  python3 tools/pmc_summary.py gpurun_out/pmc_sqd_${TAG}_$d > gpurun_out/pmc_sqd_${TAG}_$d/summary.txt
done
