#!/bin/bash
# round-5: graph launch floor, then the grouped-dW workgroup target at a rank's
# share (128 segments).  Usage: bash tools/r5_dwsweep.sh <tag>
set -o pipefail
T=${1:-r5i}
OUT=gpurun_out/$T
mkdir -p $OUT
timeout -k 10 60 ./tools/exp/graph_floor > $OUT/graph_floor.log 2>&1 || exit 1
cat $OUT/graph_floor.log
B="python -u bench.py --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline --no-host-batch"
for t in 0 128 192 256 512; do
  if [ $t -eq 0 ]; then env_=""; else env_="SMI_DWD_GROUP_TARGET=$t"; fi
  timeout -k 10 300 env $env_ $B > $OUT/l128_t$t.json 2> $OUT/l128_t$t.err || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/l128_t$t.json'))
print('target $t', d['ms_per_step'], d['kernels']['gemm_dw'], d['kernels']['gemm_splitk_reduce']['avg_ms'])"
done
