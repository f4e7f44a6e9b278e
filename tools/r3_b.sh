#!/bin/bash
# DDPG pixel tests + publish diagnosis + bench passes (one gpurun call)
tag=$1
bash tools/r3_run.sh $tag tests "tests/test_gpu_ddpg.py -k pixel" || { rc=$?; [ $rc -eq 1 ] || exit $rc; }
mkdir -p gpurun_out/$tag
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
timeout -k 10 200 python -u tools/diag_publish.py > gpurun_out/$tag/diag_publish.json 2> gpurun_out/$tag/diag_publish.err || { tail -5 gpurun_out/$tag/diag_publish.err; exit 1; }
cat gpurun_out/$tag/diag_publish.json
bash tools/r3_prof.sh $tag bench
