#!/bin/bash
# Round-5 evidence set (GPU box): the default bench line (every leg), the RE2
# and extended-rules lines, rocprofv3 kernel-trace summaries of config 2 in
# both dialects and with the extended rules, and config 2's FETCH_SIZE /
# WRITE_SIZE passes (HBM traffic per launch, tools/traffic.py).
#   tools/gpu_r5_evidence.sh TAG   -> gpurun_out/TAG/...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r5j}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
step bench_default 600 python3 -u bench.py || exit $?
step bench_re2 400 python3 -u bench.py --dialect re2 --no-batcher || exit $?
step bench_ext 400 python3 -u bench.py --extended --no-batcher || exit $?
for v in default re2 ext; do
  case $v in default) a="";; re2) a="--dialect re2";; ext) a="--extended";; esac
  step trace_$v 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace_$v -o run --output-format csv -- \
    python3 -u bench.py $a --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
done
for ctr in FETCH_SIZE WRITE_SIZE; do
  echo "== pmc $ctr" >> $OUT/steps.log
  timeout -s KILL 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_$ctr -o run --output-format csv -- \
    python3 -u bench.py --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher --no-parity > $OUT/pmc_$ctr.log 2>&1
  rc=$?; echo "pmc $ctr rc=$rc" | tee -a $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
done
python3 tools/traffic.py $OUT/pmc_FETCH_SIZE $OUT/pmc_WRITE_SIZE 2 $OUT/traffic_cfg2.json
echo "traffic rc=$?" | tee -a $OUT/steps.log
