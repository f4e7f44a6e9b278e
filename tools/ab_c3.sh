# A/B of env knobs on the C3 bench: tools/ab_c3.sh "NAME:VAR=V,VAR=V" ...
# (one bench.py per variant, 10 steps).  Output: gpurun_out/ab/<NAME>.json
set -o pipefail
mkdir -p gpurun_out/ab
cd "$GRAFT_REPO_ROOT"
for spec in "$@"; do
  name=${spec%%:*}; vars=${spec#*:}
  ( [ "$vars" != "-" ] && for kv in ${vars//,/ }; do export "$kv"; done
    timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} \
      > gpurun_out/ab/$name.json 2> gpurun_out/ab/$name.err ) || exit 1
done
