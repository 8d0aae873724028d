#!/bin/bash
# Kafka kernel phase ablations + one PMC pass (config 3).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
B="python -u bench.py --config 3 --steps 5 --warmup 2 --no-cpu-baseline"
for v in "" "--no-hits" "--diag copy" "--diag walk"; do
  timeout -k 10 300 $B $v > gpurun_out/kd.json 2> gpurun_out/kd.err; rc=$?
  [ $rc -eq 0 ] || { echo "bench $v rc=$rc"; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/kd.json')); print('$v', round(d['ms_per_step'],3), 'ms')"
done
[ "${PMC:-1}" = 1 ] && BENCH_ARGS="--config 3" PASSES=${PASSES:-tools/pmc_passes2.txt} REQS=16000000 bash tools/gpu_pmc.sh kafka
