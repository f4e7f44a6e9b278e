#!/bin/bash
# PMC passes over the HBM sweep's GAE kernels (one counter group per pass; see
# MI355X_MICROARCH.md "rocprofv3 PMC slots").  Output: gpurun_out/pmc_gae_<n>/
set -e
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
i=0
for ctrs in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS" \
            "SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_INSTS_SALU GRBM_GUI_ACTIVE" \
            "FETCH_SIZE" "WRITE_SIZE"; do
  i=$((i+1))
  timeout -s KILL 90 rocprofv3 --pmc $ctrs --output-format csv -d gpurun_out/pmc_gae_$i -o run -- python tools/bench_hbm.py --iters 3 --only "$1" > /dev/null
done
