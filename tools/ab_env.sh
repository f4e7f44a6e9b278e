#!/bin/bash
# A/B of an environment knob on one box: bench C3 alternately with VAR=A and VAR=B
# usage: bash tools/ab_env.sh OUTDIR VAR A B [rounds]
OUT=gpurun_out/$1; VAR=$2; A=$3; B=$4; R=${5:-2}
mkdir -p $OUT
for i in $(seq 1 $R); do
  for v in $A $B; do
    env $VAR=$v timeout -k 10 200 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > $OUT/c3_${VAR}_${v}_$i.json 2> $OUT/c3_${VAR}_${v}_$i.err || exit 1
  done
done
