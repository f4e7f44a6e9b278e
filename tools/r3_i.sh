#!/bin/bash
# grouped dW occupancy 3 vs 4 and workgroup target, in the C3 learn and at 128 segments
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']['gemm_dw']; print('$n', d['ms_per_step'], round(k['avg_ms']*1e3,1), k.get('tflops'))"
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_ddpg.py -k "dw_group or linear_ops" -q -x --timeout 200 > $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
SMI_LIB_VARIANT=dwgocc4 timeout -k 10 300 python -u -m pytest tests/test_gpu_ddpg.py -k "dw_group or linear_ops" -q -x --timeout 200 >> $OUT/tests.log 2>&1 || { tail -20 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
for i in 1 2; do
for v in "" dwgocc4; do
  for t in "" 1536 2048; do
    SMI_DWD_GROUP_TARGET=$t SMI_LIB_VARIANT=$v run c3_${v}_t${t}_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
  done
  SMI_LIB_VARIANT=$v run l128_${v}_$i 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
done
done
