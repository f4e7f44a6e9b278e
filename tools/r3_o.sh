#!/bin/bash
# balanced grouped-dW slabs (tail entries split): tests, trace, benches
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
[ -n "$TESTS" ] && { bash tools/r3_run.sh $tag tests "$TESTS" || exit $?; }
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for seg in 1024 128; do
  SMI_LIB_VARIANT=dwtrace timeout -k 10 120 python -u tools/bench_dwgroup.py --segments $seg > $OUT/dw_trace$seg.log 2>&1 || exit 1
  grep -v amdgpu.ids $OUT/dw_trace$seg.log
done
timeout -k 10 120 python -u tools/bench_dwgroup.py > $OUT/dw_base.log 2>&1 && grep bench $OUT/dw_base.log
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']; print('$n', d['ms_per_step'], {c: round(k[c]['avg_ms']*1e3,1) for c in ('gemm_fwd','gemm_dx','gemm_dw','gemm_reduce','lstm_fwd','lstm_bwd') if c in k})"
}
for i in 1 2; do
run c3_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_DWD_GROUP_TARGET=768 run c3_t768_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
run l128_$i 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
done
SMI_DWD_NARROW_COST=1.0 run c3_nc10 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_DWD_GROUP_TARGET=2304 run c3_t2304 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
run c4 300 python -u bench.py --config c4 --no-cpu-baseline
SMI_DWD_NARROW_COST=1.0 run l128_nc10 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
