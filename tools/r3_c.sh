#!/bin/bash
# fused-head validation: RNN / pinned / boundary / CNN / DP tests, then benches
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py tests/test_gpu_boundary.py tests/test_gpu_cnn.py tests/test_gpu_dp_pinned.py tests/test_gpu_dp_procs.py" || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
OUT=gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  cut -c1-300 $OUT/$n.json
}
run c3 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_HEAD_FUSED=0 run c3_nofuse 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
SMI_PREP_SIDE=0 run c3_l128 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
SMI_PREP_SIDE=0 SMI_HEAD_FUSED=0 run c3_l128_nofuse 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
run c5 300 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline
timeout -k 10 200 python -u tools/diag_publish.py > $OUT/diag_publish.json 2> $OUT/diag_publish.err && cat $OUT/diag_publish.json
