set -o pipefail
mkdir -p gpurun_out/r5x
for o in all head lstm; do
  timeout -k 10 120 python -u tools/bench_dwgroup.py --segments 128 --steps 25 --only $o > gpurun_out/r5x/p_$o.json 2>/dev/null || exit 1
  timeout -k 10 120 env SMI_LIB_VARIANT=dwtrace python -u tools/bench_dwgroup.py --segments 128 --steps 25 --only $o > gpurun_out/r5x/t_$o.json 2>/dev/null || exit 1
  echo "== $o"; cat gpurun_out/r5x/p_$o.json; cat gpurun_out/r5x/t_$o.json
done
