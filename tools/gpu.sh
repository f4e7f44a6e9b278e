#!/bin/bash
# One parameterised driver for the commands sent to the GPU box with gpurun
# (replaces the round-3 per-experiment r3_*.sh scripts).  Every GPU step runs
# under its own timeout and the steps stop at the first failure.
#
#   bash tools/gpu.sh <tag> tests [pytest paths/args...]   -m gpu suite (default: tests/)
#   bash tools/gpu.sh <tag> smoke                           __graft_entry__.smoke()
#   bash tools/gpu.sh <tag> bench <name> [bench.py args...] one bench line -> <name>.json
#   bash tools/gpu.sh <tag> kt <name> [bench.py args...]    rocprofv3 kernel-trace --stats of a bench command
#   bash tools/gpu.sh <tag> pmc <name> [bench.py args...]   FETCH_SIZE / WRITE_SIZE passes (separate runs)
#   bash tools/gpu.sh <tag> final                           tests + smoke + the round's bench lines + kt + pmc
#   bash tools/gpu.sh <tag> run <name> <timeout> cmd...     any command -> <name>.log (A/B arms: VAR=x env ...)
#
# Outputs go to gpurun_out/<tag>/ (copied back by gpurun); the parity report
# of the tests step is gpurun_out/<tag>/parity_report.json.
set -o pipefail
tag=$1; what=$2; shift 2
OUT=gpurun_out/$tag
mkdir -p "$OUT"
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
export TMPDIR=/tmp

die() { echo "FAILED: $*"; exit 1; }

tests() {
  local paths=${*:-tests/}
  SMI_PARITY_REPORT=$OUT/parity_report.json timeout -k 10 1000 python -u -m pytest -x -v -m gpu \
    --timeout 600 --timeout-method thread $paths > "$OUT/tests.log" 2>&1 \
    || { tail -40 "$OUT/tests.log"; die tests; }
  tail -3 "$OUT/tests.log"
}

smoke() {
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1 \
    || { tail -20 "$OUT/smoke.log"; die smoke; }
  tail -2 "$OUT/smoke.log"
}

bench() {  # name args...
  local n=$1; shift
  timeout -k 10 600 python -u bench.py "$@" > "$OUT/$n.json" 2> "$OUT/$n.err" \
    || { tail -8 "$OUT/$n.err"; die "bench $n"; }
  cut -c1-600 "$OUT/$n.json"
}

kt() {  # name args...
  local n=$1; shift
  (cd /tmp && timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv \
      -d "$ROOT/$OUT/kt_$n" -o "$n" -- python3 "$ROOT/bench.py" "$@" \
      > "$ROOT/$OUT/kt_$n.json" 2> "$ROOT/$OUT/kt_$n.err") || { tail -5 "$OUT/kt_$n.err"; die "kt $n"; }
  echo "kt $n done"
}

pmc() {  # name args...: one counter group per run (gfx950: FETCH_SIZE x2 = bytes, see MI355X guide)
  local n=$1; shift
  for c in FETCH_SIZE WRITE_SIZE; do
    (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $c --output-format csv \
        -d "$ROOT/$OUT/pmc_${n}_$c" -o run -- python3 "$ROOT/bench.py" "$@" \
        > "$ROOT/$OUT/pmc_${n}_$c.log" 2>&1) || { tail -3 "$OUT/pmc_${n}_$c.log"; die "pmc $n $c"; }
  done
  echo "pmc $n done"
}

run() {  # name timeout cmd...
  local n=$1 t=$2; shift 2
  timeout -k 10 "$t" "$@" > "$OUT/$n.log" 2>&1 || { tail -30 "$OUT/$n.log"; die "run $n"; }
  tail -5 "$OUT/$n.log"
}

case "$what" in
  tests) tests "$@" ;;
  run) run "$@" ;;
  smoke) smoke ;;
  bench) bench "$@" ;;
  kt) kt "$@" ;;
  pmc) pmc "$@" ;;
  final)
    tests
    smoke
    bench bench_default
    bench bench_c3_local128 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline
    bench bench_c5 --config c5 --steps 5 --warmup 2 --no-cpu-baseline
    bench bench_c2 --config c2 --no-cpu-baseline
    bench bench_c4 --config c4 --no-cpu-baseline
    kt c3 --config c3 --steps 10 --warmup 3 --no-cpu-baseline
    pmc c3 --config c3 --steps 5 --warmup 2 --no-cpu-baseline ;;
  *) die "unknown step $what" ;;
esac
