#!/bin/bash
# VALU recurrence with pipelined LDS chunks (vc2/vc4/vc8) + publish diagnosis
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py" || exit $?
OUT=gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for v in "" vc8 vc2; do
  SMI_LIB_VARIANT=$v timeout -k 10 120 python -u tools/bench_lstm.py --segments 128 > $OUT/lstm128_$v.json 2>&1 || exit 1
  cat $OUT/lstm128_$v.json
done
for i in 1 2; do for v in "" vc8; do
  SMI_LIB_VARIANT=$v timeout -k 10 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/l128_${v}_$i.json 2> $OUT/l128_${v}_$i.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/l128_${v}_$i.json')); k=d['kernels']; print('l128 $v', d['ms_per_step'], {c: round(k[c]['avg_ms']*1e3,1) for c in ('gemm_fwd','gemm_dx','gemm_dw','lstm_fwd','lstm_bwd') if c in k})"
done; done
timeout -k 10 300 python -u tools/diag_publish.py > $OUT/diag_publish.json 2>&1 || exit 1
cat $OUT/diag_publish.json
timeout -k 10 300 python -u tools/diag_publish.py --graph > $OUT/diag_publish_graph.json 2>&1 || exit 1
cat $OUT/diag_publish_graph.json
