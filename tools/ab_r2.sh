#!/bin/bash
# GPU tests of the GEMM paths, then an A/B of build variants on the C3 bench.
# Usage: bash tools/ab_r2.sh <tag> <variant>...   (variant 'base' = the product library)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest ${SMI_AB_TESTS:-tests/test_gpu_ddpg.py tests/test_gpu_ops.py tests/test_gpu_rnn.py tests/test_gpu_ppo.py tests/test_gpu_cnn.py tests/test_gpu_dp.py tests/test_gpu_parity_pinned.py} -k "not full_batch" -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for rep in 1 2; do
  for v in "$@"; do
    if [ "$v" = base ]; then unset SMI_LIB_VARIANT; else export SMI_LIB_VARIANT=$v; fi
    timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3_${v}_$rep.json 2>$OUT/c3_${v}_$rep.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/c3_${v}_$rep.json')); k=d['kernels']; print('$v', $rep, d['ms_per_step'], {n: round(k[n]['ms_per_step'],3) for n in ('gemm_fwd','gemm_dx','gemm_dw','lstm_fwd','lstm_bwd')})"
  done
done
if [ -f surreal_amd/libsurreal_mi_prof.so ]; then
  SMI_LIB_VARIANT=prof timeout -k 10 120 python -u tools/lstm_ticks.py > $OUT/lstm_ticks.json 2>$OUT/lstm_ticks.err && cat $OUT/lstm_ticks.json
fi
