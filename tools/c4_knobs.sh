#!/bin/bash
# C4 (DDPG, 512-row layers): split-K / panel knob sweep, interleaved
set -o pipefail
O=gpurun_out/c4knobs; mkdir -p $O
run() {  # name, env...
  local n=$1; shift
  env "$@" timeout -k 10 120 python bench.py --config c4 --steps 300 --warmup 30 --no-cpu-baseline > $O/$n.json 2>$O/$n.err || return 1
  echo "$n $(python -c "import json;d=json.loads(open('$O/$n.json').read().strip().splitlines()[-1]);print(d['ms_per_step'])")"
}
for rep in 1 2; do
  run base$rep SMI_X=0 || exit 1
  run st256_$rep SMI_SPLITK_TARGET=256 || exit 1
  run st1024_$rep SMI_SPLITK_TARGET=1024 || exit 1
  run st2048_$rep SMI_SPLITK_TARGET=2048 || exit 1
  run fsm64_$rep SMI_FWD_SPLITK_MIN=64 || exit 1
  run fsm32_st1024_$rep SMI_FWD_SPLITK_MIN=32 SMI_SPLITK_TARGET=1024 || exit 1
  run panel512_$rep SMI_PANEL_MIN_ROWS=512 || exit 1
  run nosplitfwd_$rep SMI_FWD_SPLITK_MIN=100000 || exit 1
done
