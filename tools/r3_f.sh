#!/bin/bash
# head ring-depth A/B (product depth 4 vs variants 2, 3) + head/rnn tests
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_head.py tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py" || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
OUT=gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 $t "$@" > $OUT/$n.json 2> $OUT/$n.err || { echo "FAILED $n"; tail -5 $OUT/$n.err; exit 1; }
  cut -c1-200 $OUT/$n.json
}
for i in 1 2; do
for v in "" hcd2 hcd3; do
  SMI_LIB_VARIANT=$v run c3_d${v}_$i 300 python -u bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline
  SMI_LIB_VARIANT=$v run l128_d${v}_$i 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
done
done
