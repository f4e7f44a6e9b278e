#!/bin/bash
# Round-3 evidence set on one tree: the whole -m gpu suite, smoke(), the default
# bench line (with the CPU baseline), the 128-segment rank line, then the
# kernel-trace / PMC profiles of tools/r3_prof2.sh.  Usage: bash tools/r3_final.sh <tag>
set -o pipefail
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
[ -n "$SKIP_TESTS" ] || { bash tools/r3_run.sh $tag tests tests/ || exit $?; }
bash tools/r3_run.sh $tag smoke || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { echo bench failed; tail -5 $OUT/bench_default.err; exit 1; }
cut -c1-400 $OUT/bench_default.json
timeout -k 10 300 python -u bench.py --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_local128.json 2> $OUT/bench_c3_local128.err || { echo bench128 failed; exit 1; }
timeout -k 10 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { echo bench c5 failed; exit 1; }
timeout -k 10 300 python -u bench.py --config c2 --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { echo bench c2 failed; exit 1; }
timeout -k 10 300 python -u bench.py --config c4 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err || { echo bench c4 failed; exit 1; }
echo benches ok
bash tools/r3_prof2.sh $tag
