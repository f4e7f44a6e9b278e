#!/bin/bash
# bench C3 once per value of VAR with FIXED environment FIX (e.g. SMI_DW_GROUP=1)
# usage: bash tools/ab_env2.sh OUTDIR "FIX=val ..." VAR v1 v2 ...
OUT=gpurun_out/$1; FIX=$2; VAR=$3; shift 3
mkdir -p $OUT
for v in "$@"; do
  env $FIX $VAR=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3_${VAR}_${v}.json 2> $OUT/c3_${VAR}_${v}.err || exit 1
done
