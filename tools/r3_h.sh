#!/bin/bash
# grouped dW A/B: product (64x128 tiles, 2 waves/SIMD, 4 steps in flight) vs
# dwg4 (64x64 tiles, 3 waves/SIMD) vs p8 (8 steps in flight)
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  cut -c1-200 $OUT/$n.json
}
SMI_LIB_VARIANT=dwg4 timeout -k 10 300 python -u -m pytest tests/test_gpu_ddpg.py -k "dw_group or linear_ops" -q -x --timeout 200 > $OUT/dwg4_tests.log 2>&1 || { tail -20 $OUT/dwg4_tests.log; exit 1; }
tail -2 $OUT/dwg4_tests.log
for i in 1 2; do
for v in "" dwg4 p8; do
  SMI_LIB_VARIANT=$v run dwg_${v}_$i 120 python -u tools/bench_dwgroup.py
  SMI_LIB_VARIANT=$v run dwg128_${v}_$i 120 python -u tools/bench_dwgroup.py --segments 128
  SMI_LIB_VARIANT=$v run c3_${v}_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
done
done
