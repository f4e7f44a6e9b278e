#!/bin/bash
# round 6: does measuring the clock perturb the timed region?  C3 bench arms
# interleaved: no calibration / calibration only / + in-kernel probe wave /
# + amdsmi host sampler
set -o pipefail
OUT=gpurun_out/${1:-r6c}; mkdir -p $OUT; export TMPDIR=/tmp
for rep in 1 2; do
  for arm in "nocalib:--no-calib" "none:--clock none" "probe:--clock probe" "smi:--clock smi"; do
    n=${arm%%:*}; a=${arm#*:}
    timeout -k 10 300 python -u bench.py --no-cpu-baseline --no-host-batch $a > $OUT/c3_${n}_$rep.json 2> $OUT/c3_${n}_$rep.err \
      || { tail -5 $OUT/c3_${n}_$rep.err; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/c3_${n}_$rep.json')); print('$n', $rep, d['ms_per_step'], d.get('clock'), d.get('calib_mfma_tflops'))"
  done
done
