# HBM traffic of a bench config's kernels: two rocprofv3 --pmc passes
# (FETCH_SIZE, WRITE_SIZE; MI355X_MICROARCH.md "HBM": separate passes,
# FETCH_SIZE x2 on gfx950) over a short bench.py run.
# Usage: bash tools/pmc_bench.sh [c3|c5]   Output: gpurun_out/pmc_<cfg>_{fetch,write}/
# then: python tools/pmc_traffic.py gpurun_out <cfg> > profiles/r01/pmc_traffic_<cfg>_<tag>.json
set -o pipefail
cfg=${1:-c3}
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_${cfg}_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  mkdir -p $d
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -o run -- \
    python3 bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > $d/bench.json 2> $d/err.log || exit 1
done
