# rocprofv3 kernel trace of the default bench (5 in flight) + a serial one-forward trace
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_default -o run -- python3 bench.py --steps 60 --warmup 10 > gpurun_out/prof_default.log 2>&1 && \
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_serial2 -o run -- python3 bench.py --serial --steps 20 --warmup 5 > gpurun_out/prof_serial2.log 2>&1
