# dW-kernel variants (surreal_amd/build.py VARIANTS p6/p8/occ1): per-shape dW
# timing + whole C3 learn() per variant.  Output: gpurun_out/dwd_exp/
set -o pipefail
mkdir -p gpurun_out/dwd_exp
cd "$GRAFT_REPO_ROOT"
for v in base p6 p8 occ1; do
  if [ "$v" = base ]; then unset SMI_LIB_VARIANT; else export SMI_LIB_VARIANT=$v; fi
  timeout -k 10 120 python -u tools/bench_gemm.py --only dw > gpurun_out/dwd_exp/dw_$v.jsonl 2>&1 || exit 1
  timeout -k 10 120 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/dwd_exp/c3_$v.json 2>gpurun_out/dwd_exp/c3_$v.err || exit 1
done
