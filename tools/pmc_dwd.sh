#!/bin/bash
# dW kernel stall breakdown: isolated per-shape timing + two PMC passes over
# tools/bench_gemm.py --only dw (SQ wait/active split, MFMA busy cycles).
# Output: gpurun_out/pmc_dwd/
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out/pmc_dwd
timeout -k 10 120 python -u tools/bench_gemm.py --only dw > gpurun_out/pmc_dwd/shapes.jsonl 2>&1 || exit 1
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_INSTS_SALU GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_dwd/p$i -o run -- python3 tools/bench_gemm.py --iters 3 --only dw > /dev/null || exit 1
done
