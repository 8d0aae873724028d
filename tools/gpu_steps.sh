#!/bin/bash
# Run GPU steps from a plan file, one per line: NAME SECONDS COMMAND...
# Each step has its own time limit; stdout -> gpurun_out/TAG/NAME.out,
# stderr -> NAME.err.  A pytest failure (rc 1) is recorded and the plan goes
# on; any other non-zero status (fault, abort, timeout) ends the session.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=$1; PLAN=$2
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
while read -r name secs cmd; do
  [ -z "$name" ] && continue
  case $name in \#*) continue ;; esac
  echo "== $name ($secs s): $cmd" | tee -a $OUT/steps.log
  t0=$(date +%s)
  timeout -k 10 $secs bash -c "$cmd" > $OUT/$name.out 2> $OUT/$name.err
  rc=$?
  echo "$name rc=$rc $(( $(date +%s) - t0 )) s" | tee -a $OUT/steps.log
  if [ $rc -ne 0 ] && ! { [ $rc -eq 1 ] && [[ $name == pytest* ]]; }; then
    echo "STOP after $name (rc $rc)" | tee -a $OUT/steps.log
    exit $rc
  fi
done < "$PLAN"
