#!/bin/bash
# whole-round balanced grouped dW (default) : tests + benches + trace
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
bash tools/r3_run.sh $tag tests "tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py tests/test_gpu_ddpg.py tests/test_gpu_dp_pinned.py tests/test_gpu_head.py tests/test_gpu_boundary.py" || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
SMI_LIB_VARIANT=dwtrace timeout -k 10 120 python -u tools/bench_dwgroup.py > $OUT/dw_trace1024.log 2>&1 || exit 1
grep -v amdgpu.ids $OUT/dw_trace1024.log
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']; print('$n', d['ms_per_step'], {c: round(k[c]['avg_ms']*1e3,1) for c in ('gemm_fwd','gemm_dx','gemm_dw','gemm_reduce','lstm_fwd','lstm_bwd') if c in k})"
}
for i in 1 2; do
run c3_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_DWD_ROUND_ROWS=1024 run c3_rr1024_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
done
run l128 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
run c5 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
run c5_l128 300 python -u bench.py --config c5 --local-segments 128 --steps 10 --warmup 2 --no-cpu-baseline
run c4 300 python -u bench.py --config c4 --no-cpu-baseline
