#!/bin/bash
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_cnn.py tests/test_gpu_ops.py tests/test_gpu_ddpg.py tests/test_gpu_dp_procs.py tests/test_gpu_parity_pinned.py -m gpu -x -q --timeout 900 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for a in "" "--local-segments 128"; do
  timeout -k 10 300 python -u bench.py --config c3 $a --steps 20 --warmup 3 --no-cpu-baseline > $OUT/b.json 2> $OUT/b.err || exit 1
  python -c "import json; d=json.loads(open('$OUT/b.json').read().strip().splitlines()[-1]); k=d['kernels']; print('$a', d['ms_per_step'], {n: round(k[n]['ms_per_step'],3) for n in ('gemm_fwd','gemm_dx','gemm_dw','gemm_splitk_reduce','lstm_fwd','lstm_bwd')})"
done
