#!/bin/bash
# PC sampling (rocprofv3 stochastic, beta) of one bench config:
#   bash tools/gpu_pcs.sh TAG CFG [LIB]
# -> gpurun_out/TAG/pcs_cfgN/ (per-PC samples with stall reasons).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; CFG=${2:-2}; LIB=${3:-}
OUT=gpurun_out/$TAG; mkdir -p $OUT
export TMPDIR=/tmp
[ -n "$LIB" ] && export L7M_LIB=$LIB
timeout -k 10 240 rocprofv3 --pc-sampling-beta-enabled --pc-sampling-method stochastic --pc-sampling-unit cycles \
  --pc-sampling-interval 1048576 -d $PWD/$OUT/pcs_cfg$CFG -o run --output-format csv -- \
  python3 -u bench.py --config $CFG --steps 3 --warmup 1 --no-cpu-baseline --no-e2e --no-batcher \
  > $OUT/pcs_cfg$CFG.out 2> $OUT/pcs_cfg$CFG.err
rc=$?; echo "pcs rc=$rc"; tail -3 $OUT/pcs_cfg$CFG.err; find $OUT/pcs_cfg$CFG -name "*.csv" | head; exit $rc
