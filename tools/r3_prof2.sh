#!/bin/bash
# Round-3 profiles: kernel trace of the default bench (C3) and of a 128-segment
# rank, PMC traffic (FETCH_SIZE, WRITE_SIZE) of the default bench, dW stall
# anatomy (tools/bench_dwgroup.py).  Usage: bash tools/r3_prof2.sh <tag>
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3 -o c3 -- python3 bench.py --config c3 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_c3.json 2> $OUT/kt_c3.err || { echo kt_c3 failed; tail -5 $OUT/kt_c3.err; exit 1; }
echo kt_c3 ok
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_c3l128 -o c3l128 -- python3 bench.py --config c3 --local-segments 128 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/kt_c3l128.json 2> $OUT/kt_c3l128.err || { echo kt_c3l128 failed; exit 1; }
echo kt_c3l128 ok
for k in FETCH_SIZE WRITE_SIZE; do
  d=$OUT/pmc_c3_$(echo $k | cut -d_ -f1 | tr A-Z a-z)
  mkdir -p $d
  timeout -s KILL 240 rocprofv3 --pmc $k --output-format csv -d $d -o run -- python3 bench.py --config c3 --steps 3 --warmup 1 --no-cpu-baseline > $d/bench.json 2> $d/err.log || { echo pmc $k failed; tail -3 $d/err.log; exit 1; }
  echo pmc $k ok
done
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
            "TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_BUSY_max"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d $OUT/pmcdw/p$i -o run -- python3 tools/bench_dwgroup.py --iters 5 > $OUT/pmcdw_p$i.log 2>&1 || { echo "pmc pass $i failed"; tail -3 $OUT/pmcdw_p$i.log; exit 1; }
done
echo pmcdw ok
