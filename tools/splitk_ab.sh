#!/bin/bash
# in-kernel split-K reduction: GEMM / DDPG / boundary parity, then C4 and C3 A/B
set -o pipefail
O=gpurun_out/splitk; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ddpg.py tests/test_gpu_ddpg_dp.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -2 $O/tests.log
ms() { python -c "import json;d=json.loads(open('$1').read().strip().splitlines()[-1]);print(d['ms_per_step'])"; }
for v in 1 0 1 0; do
  SMI_SPLITK_INKERNEL=$v timeout -k 10 120 python bench.py --config c4 --steps 300 --warmup 30 --no-cpu-baseline > $O/c4_$v.json 2>$O/c4_$v.err || exit 1
  echo "c4 inkernel=$v $(ms $O/c4_$v.json)"
done
for v in 1 0; do
  SMI_SPLITK_INKERNEL=$v timeout -k 10 200 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline > $O/c3_$v.json 2>$O/c3_$v.err || exit 1
  echo "c3 inkernel=$v $(ms $O/c3_$v.json)"
  SMI_SPLITK_INKERNEL=$v timeout -k 10 200 python bench.py --config c3 --local-segments 128 --steps 20 --warmup 3 --no-cpu-baseline > $O/c3l_$v.json 2>$O/c3l_$v.err || exit 1
  echo "c3 128seg inkernel=$v $(ms $O/c3l_$v.json)"
done
