#!/bin/bash
# Round-3 measurement passes.  Usage: bash tools/r3_prof.sh <tag> bench|kt|pmcdw|pmcc3
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  cut -c1-400 $OUT/$n.json
}
case "$2" in
bench)
  run c3 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
  run c3_eager 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline --graph off
  run c3_l128 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
  run c3_l128_eager 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline --graph off
  SMI_LSTM_VALU=0 run c3_l128_mfma_lstm 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
  SMI_PREP_SIDE=0 run c3_l128_noside 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
  SMI_LSTM_VALU=1 run c3_valu4 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
  run c3_l512 300 python -u bench.py --config c3 --local-segments 512 --steps 20 --warmup 3 --no-cpu-baseline
  run c3_l256 300 python -u bench.py --config c3 --local-segments 256 --steps 20 --warmup 3 --no-cpu-baseline
  run dwg 120 python -u tools/bench_dwgroup.py
  run dwg128 120 python -u tools/bench_dwgroup.py --segments 128 ;;
kt)   # kernel-trace summary of the default bench command
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3 -o c3 -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_c3.json 2> $OUT/kt_c3.err || exit 1
  timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3l128 -o c3l128 -- python3 bench.py --config c3 --local-segments 128 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_c3l128.json 2> $OUT/kt_c3l128.err || exit 1
  echo kt done ;;
pmcdw)  # stall anatomy of the grouped dW launch (tools/bench_dwgroup.py)
  i=0
  for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
              "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
              "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max"; do
    i=$((i+1))
    timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmcdw/p$i -o run -- python3 tools/bench_dwgroup.py --iters 5 > $OUT/pmcdw_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmcdw_p$i.log; exit 1; }
  done
  echo pmc done ;;
esac
