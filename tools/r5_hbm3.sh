#!/bin/bash
# round-5: GPU tests, then the in-learner HBM fractions at 65536 segments for
# each env arm given (e.g. SMI_ZF_TILE4=0 SMI_ZF_TILE4=1)
set -o pipefail
T=$1; TESTS=$2; shift 2
OUT=gpurun_out/$T; mkdir -p $OUT; export TMPDIR=/tmp
if [ "$TESTS" != "-" ]; then
  timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
      $TESTS > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -1 $OUT/tests.log
fi
for arm in "$@"; do
  timeout -k 10 600 env $arm python -u bench.py --local-segments 65536 --steps 3 --warmup 1 --no-cpu-baseline \
      --no-host-batch > $OUT/bench_c3_65536_$arm.json 2> $OUT/err_$arm.log || { tail -5 $OUT/err_$arm.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_c3_65536_$arm.json')); print('$arm', d['ms_per_step'], {k: (v.get('hbm_frac'), round(v['avg_ms']*1e3, 1)) for k, v in d['kernels'].items() if 'hbm_frac' in v})"
done
