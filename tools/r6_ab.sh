#!/bin/bash
# round 6 A/B arms on the bench (interleaved, 2 reps): r6_ab.sh <tag> <bench args> -- <arm> ...
# an arm is ENV=VALUE[,ENV=VALUE] or "base"
set -o pipefail
tag=$1; shift
args=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do args+=("$1"); shift; done
shift
OUT=gpurun_out/$tag; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for arm in "$@"; do
    envs=(); [ "$arm" != base ] && IFS=, read -ra envs <<< "$arm"
    n=$(echo "$arm" | tr '=,' '__')
    timeout -k 10 300 env "${envs[@]}" python -u bench.py "${args[@]}" --no-cpu-baseline --no-host-batch \
      > $OUT/ab_${n}_$rep.json 2> $OUT/ab_${n}_$rep.err || { tail -5 $OUT/ab_${n}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/ab_${n}_$rep.json')); k=d['kernels']
print('$arm', $rep, d['ms_per_step'], d.get('clock_mhz'), {n: round(v['avg_ms']*1e3, 2) for n, v in k.items()})"
  done
done
