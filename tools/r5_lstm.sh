#!/bin/bash
# round-5: LSTM kernels in isolation (graph-replayed launches) across A/B knobs
# (ARMS, space-separated env lists), clean and with the weights rewritten before
# every launch, then optionally the 128-segment learner bench.
# Usage: [ARMS="A=1 A=0"] bash tools/r5_lstm.sh <tag> [bench]
set -o pipefail
T=${1:-r5x}; OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -m gpu --timeout 120 --timeout-method thread \
    tests/test_gpu_rnn.py -k lstm_kernels > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for arm in ${ARMS:-SMI_LSTM_XM=1 SMI_LSTM_XM=0}; do
  for d in "" --dirty; do
    timeout -k 10 120 env ${arm//,/ } python -u tools/bench_lstm.py $d --segments ${SEGS:-128} >> $OUT/bench_lstm.log 2>&1 || { tail -5 $OUT/bench_lstm.log; exit 1; }
  done
done
python3 - $OUT/bench_lstm.log <<'PY'
import json, sys
for l in open(sys.argv[1]):
    if l.startswith('{'):
        d = json.loads(l)
        print(d['segments'], d['knobs'], 'dirty' if d['dirty'] else 'clean', d['steps'], d['fwd_us'], d['fwd_x_us'], d['bwd_us'])
PY
if [ "$2" = bench ]; then
  timeout -k 10 300 python -u bench.py --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline \
      --no-host-batch > $OUT/l128.json 2> $OUT/l128.err || { tail -5 $OUT/l128.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/l128.json')); k=d.get('kernels', {})
print('l128', d['ms_per_step'], {n: round(v['avg_ms'] * 1e3, 2) for n, v in k.items() if 'avg_ms' in v})"
fi
