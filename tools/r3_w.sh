#!/bin/bash
# statistics pass on one resident round + packed-FMA VALU recurrence: tests, A/B
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
bash tools/r3_run.sh $tag tests "tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py tests/test_gpu_dp_pinned.py tests/test_gpu_cnn.py tests/test_gpu_dp.py tests/test_gpu_ppo.py" || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "" nopk; do
  SMI_LIB_VARIANT=$v timeout -k 10 120 python -u tools/bench_lstm.py --segments 128 > $OUT/lstm128_$v.json 2>&1 || exit 1
  grep bench $OUT/lstm128_$v.json
done
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']
print('$n', d['ms_per_step'], {c: (round(k[c]['avg_ms']*1e3,1), k[c].get('hbm_frac')) for c in k if c in ('policy_rows_stats','policy_rows_grad','lstm_fwd','lstm_bwd')})"
}
for i in 1 2; do
run l128_$i 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
SMI_LIB_VARIANT=nopk run l128_nopk_$i 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
done
run c3 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
run c3_65536 600 python -u bench.py --config c3 --local-segments 65536 --steps 2 --warmup 1 --no-cpu-baseline
run c3_65536_clip 600 python -u bench.py --config c3 --ppo-mode clip --local-segments 65536 --steps 2 --warmup 1 --no-cpu-baseline
