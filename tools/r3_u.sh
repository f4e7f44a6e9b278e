#!/bin/bash
# tests touching the z-filter copies / row kernels, incl. a forced tile kernel at small B
tag=$1
[ -n "$TESTS" ] && { bash tools/r3_run.sh $tag tests "$TESTS" || exit $?; }
mkdir -p gpurun_out/$tag
OUT=gpurun_out/$tag
timeout -k 10 600 env SMI_ZF_TILE_FORCE=1 python -u -m pytest tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py -m gpu -x -q --timeout 300 > $OUT/tests_tile.log 2>&1; rc=$?; tail -3 $OUT/tests_tile.log; exit $rc
