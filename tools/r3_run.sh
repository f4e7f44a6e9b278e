#!/bin/bash
# Round-3 GPU driver.  Usage: bash tools/r3_run.sh <tag> <what> [pytest -k expr]
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "$2" in
tests)      # pytest files given in $3
  timeout -k 10 1000 python -u -m pytest $3 -m gpu --maxfail 8 -v --timeout 600 --timeout-method thread --durations=20 > $OUT/tests.log 2>&1
  rc=$?; tail -30 $OUT/tests.log; exit $rc ;;
smoke)
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
  rc=$?; tail -5 $OUT/smoke.log; exit $rc ;;
bench)      # $3: extra bench args
  timeout -k 10 400 python -u bench.py $3 > $OUT/bench.json 2> $OUT/bench.err
  rc=$?; cut -c1-600 $OUT/bench.json; tail -3 $OUT/bench.err; exit $rc ;;
esac
