#!/bin/bash
# validation of the fused heads / LSTM / publish changes, then benches
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_head.py tests/test_gpu_ops.py tests/test_gpu_ddpg.py tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py tests/test_gpu_boundary.py tests/test_gpu_cnn.py tests/test_gpu_dp_pinned.py tests/test_gpu_dp_procs.py" || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
OUT=gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  cut -c1-250 $OUT/$n.json
}
run lstm128 120 python -u tools/bench_lstm.py
SMI_LSTM_VALU=0 run lstm128_mfma 120 python -u tools/bench_lstm.py
run dwg128 120 python -u tools/bench_dwgroup.py --segments 128
SMI_DWD_GROUP_TARGET=1024 run dwg128_t1024 120 python -u tools/bench_dwgroup.py --segments 128
run dwg 120 python -u tools/bench_dwgroup.py
run c3 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_PREP_SIDE=0 run c3_noside 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_PREP_SIDE=0 run c3_l128 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
run c3_l128_side 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
timeout -k 10 200 python -u tools/diag_publish.py > $OUT/diag_publish.json 2> $OUT/diag_publish.err && cat $OUT/diag_publish.json
