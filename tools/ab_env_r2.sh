#!/bin/bash
# GPU tests of the GEMM paths, then C3 bench under environment-knob variants.
# Usage: bash tools/ab_env_r2.sh <tag> "<ENV=val ...>" ...   ("-" = defaults)
set -o pipefail
OUT=gpurun_out/$1; shift
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest ${SMI_AB_TESTS:-tests/test_gpu_ddpg.py tests/test_gpu_rnn.py} -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
i=0
for rep in 1 2; do
  for v in "$@"; do
    i=$((i+1))
    if [ "$v" = "-" ]; then envs=""; else envs="$v"; fi
    env $envs timeout -k 10 180 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3_$i.json 2>$OUT/c3_$i.err || exit 1
    python -c "import json,sys; d=json.load(open('$OUT/c3_$i.json')); k=d['kernels']; print('$v', $rep, d['ms_per_step'], {n: round(k[n]['ms_per_step'],3) for n in ('gemm_fwd','gemm_dx','gemm_dw','gemm_splitk_reduce','lstm_fwd','lstm_bwd')}, round(d['roofline']['frac'],4))"
  done
done
