#!/bin/bash
# One GPU-box pass: the -m gpu suite, then tools/bench_round.sh (C3 bench with
# CPU baseline, 2-rank gloo rehearsal, rocprofv3 kernel trace).
# Usage: bash tools/gpu_full.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -30 $OUT/gpu_tests.log; exit 1; }
tail -3 $OUT/gpu_tests.log
bash tools/bench_round.sh $1 || exit 1
cat $OUT/bench_c3.json
