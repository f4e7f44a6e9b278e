#!/bin/bash
# last round-2 pass on the final tree: full GPU suite + smoke, C3 bench line, Adam/gather HBM sweep
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 1100 python -u -m pytest tests -m gpu -q --timeout 900 --timeout-method thread > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
tail -2 $OUT/gpu_tests.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python -u bench.py > $OUT/bench_c3.json 2> $OUT/bench_c3.err || exit 1
cut -c1-400 $OUT/bench_c3.json
timeout -k 10 200 python -u bench.py --config c4 > $OUT/bench_c4.json 2> $OUT/bench_c4.err || exit 1
cut -c1-300 $OUT/bench_c4.json
timeout -k 10 200 python -u tools/bench_hbm.py --iters 20 --only adam_clip,gather_rows > $OUT/hbm_adam_gather.jsonl 2> $OUT/hbm.err || exit 1
cat $OUT/hbm_adam_gather.jsonl | cut -c1-200
