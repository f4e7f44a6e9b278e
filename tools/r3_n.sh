#!/bin/bash
# grouped-dW workgroup clock trace (bench_dwgroup, C3 rows and one rank's rows)
tag=$1
OUT=gpurun_out/$tag
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 120 python -u tools/bench_dwgroup.py > $OUT/dw_base.log 2>&1 || exit 1
cat $OUT/dw_base.log
SMI_LIB_VARIANT=dwtrace timeout -k 10 120 python -u tools/bench_dwgroup.py > $OUT/dw_trace.log 2>&1 || { tail -5 $OUT/dw_trace.log; exit 1; }
cat $OUT/dw_trace.log
SMI_LIB_VARIANT=dwtrace timeout -k 10 120 python -u tools/bench_dwgroup.py --segments 128 > $OUT/dw_trace128.log 2>&1 || exit 1
cat $OUT/dw_trace128.log
