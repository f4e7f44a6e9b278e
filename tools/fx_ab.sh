set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_rnn.py tests/test_gpu_cnn.py tests/test_gpu_dp_procs.py > gpurun_out/fx_tests.log 2>&1 && \
timeout -k 10 200 python -u bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/fx_c3_on.json 2> gpurun_out/fx_err2.log && \
timeout -k 10 200 python -u bench.py --config c5 --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/fx_c5_on.json 2> gpurun_out/fx_err4.log
