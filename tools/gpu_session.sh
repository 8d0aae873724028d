#!/bin/bash
# One GPU session: run the named steps in order, each under its own time
# limit; the first fatal exit (crash, abort, timeout) ends the session.
#   tools/gpu_session.sh TAG step...   steps: tests | tests:<pytest -k expr> |
#   bench:<cfg> | prof:<cfg> | pmc:<cfg>:<COUNTER> | smoke
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
step() {  # name, seconds, command...
  local name=$1 secs=$2; shift 2
  echo "== $name: $*" >> $OUT/steps.log
  timeout -k 10 $secs "$@" > $OUT/$name.out 2> $OUT/$name.err
  local rc=$?; echo "$name rc=$rc" | tee -a $OUT/steps.log; return $rc
}
for s in "$@"; do
  case $s in
    tests) step pytest_gpu 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread
           rc=$?; [ $rc -le 1 ] || exit $rc ;;
    tests:*) step pytest_sel 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "${s#tests:}"
           rc=$?; [ $rc -le 1 ] || exit $rc ;;
    smoke) step smoke 300 python -u -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench:*) step bench_${s#bench:} 600 python -u bench.py --config ${s#bench:} || exit $? ;;
    benchq:*) step benchq_${s#benchq:} 600 python -u bench.py --config ${s#benchq:} --no-cpu-baseline || exit $? ;;
    prof:*) c=${s#prof:}; step prof_$c 600 rocprofv3 --kernel-trace --stats -d $PWD/$OUT/prof_$c -o run --output-format csv -- python3 -u bench.py --config $c --steps 20 --warmup 2 --no-cpu-baseline --no-e2e --no-batcher || exit $? ;;
    pmc:*) c=${s#pmc:}; cfg=${c%%:*}; ctr=${c#*:}
           step pmc_${cfg}_$ctr 300 rocprofv3 --pmc $ctr -d $PWD/$OUT/pmc_${cfg}_$ctr -o run --output-format csv -- python3 -u bench.py --config $cfg --steps 1 --warmup 0 --no-cpu-baseline --no-e2e --no-batcher || exit $? ;;
    vtests:*) v=${s#vtests:}; name=${v%%:*}; kx=${v#*:}
           L7M_LIB=variants/$name.so step vtests_$name 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread -k "$kx"
           rc=$?; [ $rc -le 1 ] || exit $rc ;;
    diag:*) v=${s#diag:}; cfg=${v%%:*}; mode=${v#*:}
           step diag_${cfg}_$mode 300 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline --diag $mode || exit $? ;;
    envb:*) v=${s#envb:}; name=${v%%:*}; rest=${v#*:}; cfg=${rest%%:*}; kv=${rest#*:}
           step envb_${name}_$cfg 300 env $kv python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline || exit $? ;;
    bargs:*) v=${s#bargs:}; name=${v%%:*}; rest=${v#*:}; cfg=${rest%%:*}; extra=${rest#*:}
           step bargs_${name}_$cfg 300 python -u bench.py --config $cfg --steps 10 --warmup 2 --no-cpu-baseline ${extra//,/ } || exit $? ;;
    var:*) v=${s#var:}; name=${v%%:*}; cfg=${v#*:}
           L7M_LIB=variants/$name.so step var_${name}_$cfg 300 python -u bench.py --config $cfg --steps 5 --warmup 2 --no-cpu-baseline || exit $? ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
