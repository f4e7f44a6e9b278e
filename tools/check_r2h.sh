#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_ppo.py tests/test_gpu_cnn.py tests/test_gpu_dp.py tests/test_gpu_dp_procs.py tests/test_gpu_parity_pinned.py -k "not c5_full" -m gpu -x -q --timeout 900 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 1
python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print(d['ms_per_step'], d['value'])"
bash tools/final_r2.sh $1 prof || exit 1
