#!/bin/bash
# Remaining GPU tests after the C5 pinned case, then tools/bench_round.sh.
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1000 python -u -m pytest tests/test_gpu_parity_pinned.py tests/test_gpu_ppo.py tests/test_gpu_rnn.py -k "c5 or host_path or staging or test_gpu_ppo or test_gpu_rnn" -m gpu -x -v --timeout 120 --timeout-method thread --durations=10 > $OUT/gpu_tests_rest.log 2>&1 || { tail -30 $OUT/gpu_tests_rest.log; exit 1; }
tail -15 $OUT/gpu_tests_rest.log
bash tools/bench_round.sh $1 || exit 1
cat $OUT/bench_c3.json
