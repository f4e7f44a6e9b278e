#!/bin/bash
# DDPG grouped weight gradients: parity tests, then C4 bench with / without grouping
set -o pipefail
O=gpurun_out/ddpg_grp; mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread \
  tests/test_gpu_ddpg.py tests/test_gpu_ddpg_dp.py tests/test_gpu_boundary.py > $O/tests.log 2>&1 || { tail -30 $O/tests.log; exit 1; }
tail -3 $O/tests.log
for v in 1 0 1 0; do
  SMI_DDPG_DW_GROUP=$v timeout -k 10 180 python bench.py --config c4 --steps 200 --warmup 20 > $O/c4_g$v.json 2>$O/c4_g$v.err || exit 1
  echo "group=$v $(python -c "import json;d=json.loads(open('$O/c4_g$v.json').read().strip().splitlines()[-1]);print(d['value'],d['ms_per_step'])")"
done
