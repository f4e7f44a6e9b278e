#!/bin/bash
# policy statistics row pass with the next row prefetched: C3 and 65536 segments
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']
print('$n', d['ms_per_step'], {c: (round(k[c]['avg_ms']*1e3,1), k[c].get('hbm_frac')) for c in k if c in ('policy_rows_stats','policy_rows_grad','value_rows','zf_tmajor')})"
}
[ -n "$TESTS" ] && { bash tools/r3_run.sh $tag tests "$TESTS" || exit $?; }
run c3 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
run c3_65536 600 python -u bench.py --config c3 --local-segments 65536 --steps 2 --warmup 1 --no-cpu-baseline
run c3_65536_clip 600 python -u bench.py --config c3 --ppo-mode clip --local-segments 65536 --steps 2 --warmup 1 --no-cpu-baseline
