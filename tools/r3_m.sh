#!/bin/bash
# publish: D2H issued after the learner's post-publish host reads
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u tools/diag_publish.py > $OUT/diag_publish.json 2>&1 || exit 1
cat $OUT/diag_publish.json
timeout -k 10 300 python -u tools/diag_publish.py --graph > $OUT/diag_publish_graph.json 2>&1 || exit 1
cat $OUT/diag_publish_graph.json
bash tools/r3_run.sh $tag tests "tests/test_gpu_boundary.py"
# grouped-dW anatomy: product / MFMAs only / operand stream only (kernel trace)
for v in "" dwdiag_mfma dwdiag_load; do
  d=$OUT/dw_${v:-base}
  SMI_LIB_VARIANT=$v timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $d -o run -- python3 tools/bench_dwgroup.py --iters 30 > $d.log 2>&1 || { echo dw $v failed; tail -3 $d.log; exit 1; }
  tail -1 $d.log
done
# the 128-segment rank eager (ranks > 1 run eager) vs graph replay
for g in on off; do
  timeout -k 10 300 python -u bench.py --config c3 --local-segments 128 --graph $g --steps 20 --warmup 3 --no-cpu-baseline > $OUT/l128_graph_$g.json 2> $OUT/l128_graph_$g.err || exit 1
  python3 -c "import json; d=json.load(open('$OUT/l128_graph_$g.json')); print('l128 graph $g', d['ms_per_step'])"
done
