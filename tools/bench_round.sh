#!/bin/bash
# One GPU-box pass: C3 bench (N=1, with CPU baseline), a 2-rank gloo rehearsal
# of the data-parallel launch on one GPU, and a rocprofv3 kernel trace of C3.
# Usage: bash tools/bench_round.sh <outdir under gpurun_out>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
SMI_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c3_dp2_gloo.json 2> $OUT/bench_c3_dp2_gloo.err || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c3 -o c3 -- python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_c3.json 2> $OUT/prof_c3.err || exit 1
