#!/bin/bash
# r4 LSTM forward with the x sequence staged in LDS: tests + benches
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_head.py tests/test_gpu_parity_pinned.py tests/test_gpu_rnn.py tests/test_gpu_cnn.py" || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
OUT=gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  [ "$n" = lstm1024 ] && { cat $OUT/$n.json; return; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']; print('$n', d['ms_per_step'], {c: round(k[c]['avg_ms']*1e3,1) for c in ('gemm_fwd','gemm_dx','gemm_dw','lstm_fwd','lstm_bwd') if c in k})"
}
for i in 1 2; do
run c3_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
run l128_$i 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
done
run c5 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
run c5_l128 300 python -u bench.py --config c5 --local-segments 128 --steps 10 --warmup 2 --no-cpu-baseline
run lstm1024 120 python -u tools/bench_lstm.py --segments 1024 || true
