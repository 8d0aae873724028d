#!/bin/bash
# Time the in-tree library and every variants/*.so on one bench config.
# usage: CFG=3 bash tools/gpu_variants.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in cilium_amd/libl7match.so variants/*.so; do
  L7M_LIB=$L timeout -k 10 200 python -u bench.py --config ${CFG:-3} --steps 5 --warmup 2 --no-cpu-baseline \
    > gpurun_out/var.json 2> gpurun_out/var.err; rc=$?
  [ $rc -eq 0 ] || { echo "$L rc=$rc"; exit $rc; }
  python -c "import json; d=json.load(open('gpurun_out/var.json')); print('$L', round(d['ms_per_step'], 3))"
done
