#!/bin/bash
# round-5: tests + 128-segment and C3 A/B of one env knob (ARM)
set -o pipefail
T=$1; ARM=$2; TESTS=${3:-"tests/test_gpu_rnn.py tests/test_gpu_parity_pinned.py tests/test_gpu_dp_pinned.py tests/test_gpu_dp.py"}
bash tools/r5_ab.sh $T "$TESTS" "--local-segments 128 --steps 20 --warmup 3" "$ARM" "" && \
bash tools/r5_ab.sh ${T}c3 - "--steps 20 --warmup 3" "$ARM" ""
