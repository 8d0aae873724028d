#!/bin/bash
# Round-6 evidence set (GPU box), the final build: the GPU suite as the driver
# runs it, a bench line for every BASELINE configuration (1, 2 default with
# every leg, 3, 4 on two gloo ranks, 5) plus the RE2 and extended-rules
# lines, rocprofv3 kernel-trace summaries of the same runs, FETCH_SIZE /
# WRITE_SIZE passes (tools/traffic.py) for configs 2, 3 and 5.
#   tools/gpu_r6_evidence.sh TAG [part]   -> gpurun_out/TAG/...
# part: all (default) | pmc | bench1 | bench2 | trace (one gpurun call each; pmc first, so
# that the bench lines find the traffic of their own device code)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-r6e}; PART=${2:-all}
OUT=gpurun_out/$TAG; mkdir -p $OUT; export TMPDIR=/tmp
step() { local name=$1 secs=$2; shift 2; echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err; local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc; }
if [ "$PART" = all ] || [ "$PART" = bench1 ]; then
  step gpu_suite 900 python3 -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread || exit $?
  step bench_cfg2 700 python3 -u bench.py || exit $?
  step bench_cfg1 400 python3 -u bench.py --config 1 || exit $?
  step bench_cfg3 600 python3 -u bench.py --config 3 || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = bench2 ]; then
  step bench_cfg5 600 python3 -u bench.py --config 5 --no-e2e || exit $?
  step bench_re2 400 python3 -u bench.py --dialect re2 --no-batcher --no-e2e || exit $?
  step bench_ext 400 python3 -u bench.py --extended --no-batcher --no-e2e || exit $?
  step bench_cfg4 900 python3 -u -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port 29517 bench.py --config 4 --gpus 2 --backend gloo --no-cpu-baseline --no-e2e --no-batcher || exit $?
  step bench_cfg4_n1 600 python3 -u bench.py --config 4 --no-e2e || exit $?
  step batcher_solo 120 cilium_amd/batcher_bench 2 1000000 3 1 8 || exit $?
fi
if [ "$PART" = all ] || [ "$PART" = trace ]; then
  for v in cfg2 cfg1 cfg3 cfg5 re2 ext; do
    case $v in cfg2) a="";; cfg1) a="--config 1";; cfg3) a="--config 3";; cfg5) a="--config 5";;
               re2) a="--dialect re2";; ext) a="--extended";; esac
    step trace_$v 400 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/trace_$v -o run --output-format csv -- \
      python3 -u bench.py $a --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher --no-parity || exit $?
  done
fi
if [ "$PART" = all ] || [ "$PART" = pmc ]; then
  for cfg in 2 3 5; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      echo "== pmc $ctr cfg$cfg" >> $OUT/steps.log
      timeout -s KILL 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_${ctr}_$cfg -o run --output-format csv -- \
        python3 -u bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher --no-parity \
        > $OUT/pmc_${ctr}_$cfg.log 2>&1
      rc=$?; echo "pmc $ctr cfg$cfg rc=$rc" | tee -a $OUT/steps.log; [ $rc -eq 0 ] || exit $rc
    done
    python3 tools/traffic.py $OUT/pmc_FETCH_SIZE_$cfg $OUT/pmc_WRITE_SIZE_$cfg $cfg $OUT/traffic_cfg$cfg.json
    echo "traffic cfg$cfg rc=$?" | tee -a $OUT/steps.log
  done
fi
