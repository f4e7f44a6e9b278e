#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_cnn.py tests/test_gpu_dp_procs.py tests/test_gpu_parity_pinned.py -k "not full_batch" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
timeout -k 10 300 python -u bench.py --config c3 --local-segments 65536 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c3_local65536.json 2> $OUT/bench_c3_local65536.err || exit 1
python - <<'PY'
import json,sys
for f in ['bench_c3','bench_c3_local65536']:
    d=json.load(open(f'gpurun_out/'+sys.argv[1] if False else f'$OUT/{f}.json')); k=d['kernels']
    print(f, d['ms_per_step'], {n:(round(k[n]['avg_ms']*1e3,1), k[n].get('hbm_frac')) for n in ('policy_rows_stats','policy_rows_grad','value_rows')})
PY
