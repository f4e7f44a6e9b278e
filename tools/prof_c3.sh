set -o pipefail
mkdir -p gpurun_out/prof_c3
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o c3 -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > gpurun_out/prof_c3/bench.json 2> gpurun_out/prof_c3/err.log
