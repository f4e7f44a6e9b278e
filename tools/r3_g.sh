#!/bin/bash
# new 128-segment fixture cases + LSTM recurrence form A/B at 1024 segments
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_parity_pinned.py tests/test_gpu_rnn.py tests/test_gpu_head.py" || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
OUT=gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  cut -c1-200 $OUT/$n.json
}
run lstm1024_mfma 120 python -u tools/bench_lstm.py --segments 1024
SMI_LSTM_VALU_R=1 run lstm1024_r1 120 python -u tools/bench_lstm.py --segments 1024
SMI_LSTM_VALU_R=2 run lstm1024_r2 120 python -u tools/bench_lstm.py --segments 1024
SMI_LSTM_VALU_R=4 run lstm1024_r4 120 python -u tools/bench_lstm.py --segments 1024
run lstm128 120 python -u tools/bench_lstm.py
run c3 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_LSTM_VALU_R=2 run c3_r2 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_LSTM_VALU_R=1 run c3_r1 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
run c3_l128 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
run c3_l256 300 python -u bench.py --config c3 --local-segments 256 --steps 20 --warmup 3 --no-cpu-baseline
SMI_LSTM_VALU_R=1 run c3_l256_r1 300 python -u bench.py --config c3 --local-segments 256 --steps 20 --warmup 3 --no-cpu-baseline
run c3_l512 300 python -u bench.py --config c3 --local-segments 512 --steps 20 --warmup 3 --no-cpu-baseline
SMI_LSTM_VALU_R=2 run c3_l512_r2 300 python -u bench.py --config c3 --local-segments 512 --steps 20 --warmup 3 --no-cpu-baseline
