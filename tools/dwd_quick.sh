set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ddpg.py > gpurun_out/dwd_tests.log 2>&1 && \
timeout -k 10 120 python -u tools/bench_gemm.py --only dw > gpurun_out/dwd_on.jsonl 2>&1 && \
SMI_SPLITK_TARGET=1024 timeout -k 10 120 python -u tools/bench_gemm.py --only dw > gpurun_out/dwd_on1024.jsonl 2>&1 && \
SMI_SPLITK_TARGET=256 timeout -k 10 120 python -u tools/bench_gemm.py --only dw > gpurun_out/dwd_on256.jsonl 2>&1
