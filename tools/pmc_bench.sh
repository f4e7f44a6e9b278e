# HBM traffic of the C3 bench's kernels: two rocprofv3 --pmc passes (FETCH_SIZE,
# WRITE_SIZE; MI355X_MICROARCH.md "HBM": separate passes, FETCH_SIZE x2 on
# gfx950) over a short bench.py run, then the kernel-trace stats pass.
# Output: gpurun_out/pmc_bench_{fetch,write}/, gpurun_out/prof_c3/
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
for c in FETCH_SIZE WRITE_SIZE; do
  d=gpurun_out/pmc_bench_$(echo $c | cut -d_ -f1 | tr A-Z a-z)
  mkdir -p $d
  timeout -s KILL 240 rocprofv3 --pmc $c --output-format csv -d $d -o run -- \
    python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > $d/bench.json 2> $d/err.log || exit 1
done
bash tools/prof_c3.sh
