#!/bin/bash
# round-5: in-learner HBM fractions at 65536 segments (231 MB row passes),
# A/B of the statistics pass form (SMI_STATS_LEAN), then its parity tests
set -o pipefail
OUT=gpurun_out/${1:-r5ap}; mkdir -p $OUT; export TMPDIR=/tmp
for arm in SMI_STATS_LEAN=0 SMI_STATS_LEAN=1; do
  timeout -k 10 600 env $arm python -u bench.py --local-segments 65536 --steps 3 --warmup 1 --no-cpu-baseline \
      --no-host-batch > $OUT/bench_c3_65536_$arm.json 2> $OUT/err_$arm.log || { tail -5 $OUT/err_$arm.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/bench_c3_65536_$arm.json')); print('$arm', d['ms_per_step'], {k: (v.get('hbm_frac'), round(v['avg_ms']*1e3, 1)) for k, v in d['kernels'].items() if 'hbm_frac' in v})"
done
timeout -k 10 600 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread \
    tests/test_gpu_parity_pinned.py tests/test_gpu_rnn.py tests/test_gpu_dp_pinned.py > $OUT/tests.log 2>&1; tail -1 $OUT/tests.log
