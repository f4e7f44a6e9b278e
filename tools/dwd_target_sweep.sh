#!/bin/bash
# dW split-K target sweep (SMI_DWD_TARGET = workgroups per dW launch):
# isolated per-shape timing, then whole C3 learn() for each target.
# Output: gpurun_out/dwd_sweep/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/dwd_sweep
for t in 128 192 240 256 320 384 512; do
  SMI_DWD_TARGET=$t timeout -k 10 120 python -u tools/bench_gemm.py --only dw > gpurun_out/dwd_sweep/dw_$t.jsonl 2>&1 || exit 1
done
for t in 256 192 384 512 256; do
  SMI_DWD_TARGET=$t timeout -k 10 120 python -u bench.py --steps 20 --warmup 3 --no-cpu-baseline > gpurun_out/dwd_sweep/c3_$t.json 2>gpurun_out/dwd_sweep/c3_$t.err || exit 1
  cp gpurun_out/dwd_sweep/c3_$t.json gpurun_out/dwd_sweep/c3_${t}_$RANDOM.json
done
