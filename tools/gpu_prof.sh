#!/bin/bash
# rocprofv3 kernel-trace summaries of configs 2, 3 and 4 (20 timed + 2 warmup launches each).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${1:-prof}
mkdir -p $OUT
export TMPDIR=/tmp
for cfg in 2 3 4; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/cfg$cfg -o run --output-format csv -- \
    python3 -u bench.py --config $cfg --steps 20 --warmup 2 --no-cpu-baseline > $OUT/cfg$cfg.json 2> $OUT/cfg$cfg.err
  rc=$?; echo "cfg$cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
