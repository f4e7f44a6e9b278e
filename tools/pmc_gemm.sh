#!/bin/bash
# PMC passes over tools/bench_gemm.py (one counter group per pass, see
# MI355X_MICROARCH.md "rocprofv3 PMC slots").  Output: gpurun_out/pmc_gemm_<n>/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS GRBM_GUI_ACTIVE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_gemm_$i -o run -- python tools/bench_gemm.py --iters 3 ${1:+--only $1} > /dev/null
done
