# Counter passes (one rocprofv3 --pmc run each, within the per-block limits of
# MI355X_MICROARCH.md) over a short bench.py run; summarise with
#   python tools/pmc_summary.py gpurun_out/<tag>/pmc_*
# Usage: bash tools/pmc_rows.sh <tag> [bench.py args...]
set -o pipefail
tag=$1; shift
ROOT=${GRAFT_REPO_ROOT:-$(pwd)}
OUT=$ROOT/gpurun_out/$tag
mkdir -p "$OUT"
export TMPDIR=/tmp
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_VMEM_RD"
P2="SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TA_BUSY_avr GRBM_GUI_ACTIVE"
i=0
for P in "$P1" "$P2" FETCH_SIZE WRITE_SIZE; do
  i=$((i + 1))
  (cd /tmp && timeout -s KILL 300 rocprofv3 --pmc $P --output-format csv -d "$OUT/pmc_p$i" -o run -- \
      python3 "$ROOT/bench.py" "$@" > "$OUT/pmc_p$i.log" 2>&1) || { tail -5 "$OUT/pmc_p$i.log"; exit 1; }
  echo "pass $i done"
done
