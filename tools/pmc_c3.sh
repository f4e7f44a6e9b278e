#!/bin/bash
# PMC passes over the C3 learner (tools/time_c3.py); one counter group per pass
# (MI355X_MICROARCH.md "rocprofv3 PMC slots").  Output: gpurun_out/pmc_c3_<n>/
set -e
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU SQ_INSTS_MFMA GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_c3_$i -o run -- python tools/time_c3.py ${1:-1024} > /dev/null
done
