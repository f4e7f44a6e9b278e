#!/bin/bash
# Round-2 evidence pass.  Usage: bash tools/final_r2.sh <tag> tests|bench|prof
set -o pipefail
OUT=gpurun_out/$1
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
case "$2" in
tests)
  timeout -k 10 1100 python -u -m pytest tests -m gpu -x -v --timeout 900 --timeout-method thread --durations=15 > $OUT/gpu_tests.log 2>&1 || { tail -40 $OUT/gpu_tests.log; exit 1; }
  tail -20 $OUT/gpu_tests.log
  timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 1; }
  tail -3 $OUT/smoke.log ;;
bench)
  for c in c3 c5 c2 c4; do
    timeout -k 10 300 python -u bench.py --config $c --steps 20 --warmup 3 > $OUT/bench_$c.json 2> $OUT/bench_$c.err || exit 1
    cut -c1-300 $OUT/bench_$c.json
  done
  timeout -k 10 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_local128.json 2> $OUT/bench_c3_local128.err || exit 1
  SMI_PANEL_MIN_ROWS=4096 timeout -k 10 300 python -u bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c3_local128_nopanel.json 2> $OUT/bench_c3_local128_nopanel.err || exit 1
  timeout -k 10 300 python -u bench.py --config c5 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $OUT/bench_c5_local128.json 2> $OUT/bench_c5_local128.err || exit 1
  # streaming kernels at > 256 MB working sets inside learn(): 65536 segments
  timeout -k 10 300 python -u bench.py --config c3 --local-segments 65536 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/bench_c3_local65536.json 2> $OUT/bench_c3_local65536.err || exit 1
  SMI_DIST_BACKEND=gloo timeout -k 10 300 python -u bench.py --gpus 2 --steps 10 --warmup 2 --no-cpu-baseline > $OUT/bench_c3_dp2_gloo.json 2> $OUT/bench_c3_dp2_gloo.err || exit 1
  timeout -k 10 300 python -u tools/bench_hbm.py --iters 20 > $OUT/hbm_sweep.jsonl 2> $OUT/hbm_sweep.err || exit 1
  cut -c1-200 $OUT/hbm_sweep.jsonl
  cut -c1-300 $OUT/bench_c3_local128.json ;;
prof)
  for c in c3 c5; do
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$c -o $c -- python3 bench.py --config $c --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof_$c.json 2> $OUT/prof_$c.err || exit 1
  done
  for c in c3 c5; do
    for k in FETCH_SIZE WRITE_SIZE; do
      d=$OUT/pmc_${c}_$(echo $k | cut -d_ -f1 | tr A-Z a-z)
      mkdir -p $d
      timeout -s KILL 240 rocprofv3 --pmc $k --output-format csv -d $d -o run -- python3 bench.py --config $c --steps 3 --warmup 1 --no-cpu-baseline > $d/bench.json 2> $d/err.log || exit 1
    done
  done
  echo prof done ;;
esac
