#!/bin/bash
# round-5 GPU check: the LSTM harness, then the whole -m gpu suite WITHOUT -x
# (every failure listed), then the bench lines.  Usage: bash tools/r5_tests.sh <tag>
set -o pipefail
T=${1:-r5x}
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 60 ./tools/exp/lstm_v_exp > $OUT/lstm_v_exp.log 2>&1 || { echo "harness failed"; exit 1; }
grep -v ticks $OUT/lstm_v_exp.log
SMI_PARITY_REPORT=$OUT/parity_report.json timeout -k 10 1100 python -u -m pytest -v -m gpu \
    --timeout 600 --timeout-method thread tests/ > $OUT/tests.log 2>&1
rc=$?
tail -15 $OUT/tests.log
[ $rc -eq 0 ] || [ $rc -eq 1 ] || { echo "pytest aborted rc=$rc"; exit 1; }
timeout -k 10 600 python -u bench.py --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/l128.json 2> $OUT/l128.err || exit 1
cut -c1-400 $OUT/l128.json
timeout -k 10 600 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err || exit 1
cut -c1-400 $OUT/c3.json
