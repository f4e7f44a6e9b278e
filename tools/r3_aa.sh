#!/bin/bash
# head backward with dH1 over dH2 (three workgroups per CU at RT = 2)
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
bash tools/r3_run.sh $tag tests "tests/test_gpu_head.py tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py tests/test_gpu_cnn.py" || exit $?
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/$n.json')); k=d['kernels']
print('$n', d['ms_per_step'], {c: round(k[c]['avg_ms']*1e3,1) for c in k if c in ('lstm_fwd','lstm_bwd','gemm_fwd','gemm_dx','gemm_dw')})"
}
for i in 1 2; do
run c3_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
done
run l128 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
run c5 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
