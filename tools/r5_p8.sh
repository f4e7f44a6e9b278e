set -o pipefail
mkdir -p gpurun_out/r5y
for o in all lstm; do
  for v in "" p8; do
    timeout -k 10 120 env SMI_LIB_VARIANT=$v python -u tools/bench_dwgroup.py --segments 128 --steps 25 --only $o 2>/dev/null | sed "s/^/$o [$v] /" || exit 1
  done
done
bash tools/r5_ab.sh r5y - "--local-segments 128 --steps 20 --warmup 3" "" "SMI_LIB_VARIANT=p8"
