set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_ddpg.py > gpurun_out/panel_tests.log 2>&1 && \
SMI_PANEL=0 timeout -k 10 120 python -u tools/bench_gemm.py --only fwd,dx > gpurun_out/panel_off.jsonl 2>&1 && \
timeout -k 10 120 python -u tools/bench_gemm.py --only fwd,dx > gpurun_out/panel_on.jsonl 2>&1 && \
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rnn.py tests/test_gpu_cnn.py tests/test_gpu_ppo.py >> gpurun_out/panel_tests.log 2>&1 && \
SMI_PANEL=0 timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/panel_c3_off.json 2> gpurun_out/panel_err1.log && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/panel_c3_on.json 2> gpurun_out/panel_err2.log && \
timeout -k 10 200 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/panel_c5_on.json 2> gpurun_out/panel_err4.log
