# PMC passes (one rocprofv3 run per counter group) over tools/run_c2.py, plus
# the phase timer of the noinline variant.  Run on the GPU box from the repo root:
#   bash tools/pmc_fused.sh
set -e
mkdir -p gpurun_out/pmc
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_INST_ANY SQ_WAIT_ANY SQ_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_SMEM -d $R/gpurun_out/pmc/p1 -o p1 --output-format csv -- python3 $R/tools/run_c2.py 10 > $R/gpurun_out/pmc/p1.log 2>&1
timeout -k 10 120 rocprofv3 --pmc SQC_ICACHE_REQ SQC_ICACHE_HITS SQC_ICACHE_MISSES SQ_IFETCH -d $R/gpurun_out/pmc/p2 -o p2 --output-format csv -- python3 $R/tools/run_c2.py 10 > $R/gpurun_out/pmc/p2.log 2>&1
cd $R
timeout -k 10 200 python -u tools/fused_breakdown.py --phases --variant=noinl > gpurun_out/phases_noinl.log 2>&1
timeout -k 10 200 python -u tools/fused_breakdown.py --variant=noinl > gpurun_out/bd_noinl.log 2>&1
