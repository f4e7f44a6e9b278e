#!/bin/bash
# round-5 A/B: optional test paths, then interleaved bench arms.
#   bash tools/r5_ab.sh <tag> "<pytest paths or ->" "<bench args>" ARM1 ARM2 ...
# each ARM is an env assignment list ("" = default), e.g. "SMI_LSTM_XM=0";
# arms run twice, interleaved (A B A B), one JSON line each.
set -o pipefail
T=$1; TESTS=$2; BARGS=$3; shift 3
OUT=gpurun_out/$T
mkdir -p $OUT
export TMPDIR=/tmp
if [ "$TESTS" != "-" ]; then
  SMI_PARITY_REPORT=$OUT/parity_report.json timeout -k 10 900 python -u -m pytest -x -v -m gpu \
      --timeout 300 --timeout-method thread $TESTS > $OUT/tests.log 2>&1
  rc=$?
  tail -4 $OUT/tests.log
  [ $rc -eq 0 ] || { grep -E "FAIL|Error" $OUT/tests.log | head -20; exit 1; }
fi
for rep in 1 2; do
  i=0
  for arm in "$@"; do
    i=$((i + 1))
    timeout -k 10 300 env $arm python -u bench.py $BARGS --no-cpu-baseline --no-host-batch \
        > $OUT/arm${i}_$rep.json 2> $OUT/arm${i}_$rep.err || { tail -5 $OUT/arm${i}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/arm${i}_$rep.json')); k=d.get('kernels', {})
print('arm $i [$arm] rep $rep', d['ms_per_step'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in k.items() if 'avg_ms' in v})"
  done
done
