#!/bin/bash
set -o pipefail
OUT=gpurun_out/${1:-r5aq}; mkdir -p $OUT; export TMPDIR=/tmp
timeout -k 10 600 python -u bench.py --local-segments 65536 --steps 3 --warmup 1 --no-cpu-baseline \
    --no-host-batch > $OUT/bench_c3_65536.json 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
python3 -c "
import json; d=json.load(open('$OUT/bench_c3_65536.json')); print(d['ms_per_step'], {k: (v.get('hbm_frac'), round(v['avg_ms']*1e3, 1)) for k, v in d['kernels'].items() if 'hbm_frac' in v})"
bash tools/r5_ab.sh ${1:-r5aq}t "tests/test_gpu_parity_pinned.py tests/test_gpu_rnn.py tests/test_gpu_dp_pinned.py tests/test_gpu_negative_controls.py" "--steps 20 --warmup 3" ""
