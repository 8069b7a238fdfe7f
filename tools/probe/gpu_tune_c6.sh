# conv table tuned under 6-way concurrency vs the shipped 4-way one, bench at 5 and 6 in flight
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m mlmicroservicetemplate_amd.ops.autotune --concurrency 6 --no-torch --out gpurun_out/tune_c6.json > gpurun_out/tune_c6.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench_c4_if5.log 2>&1 && \
MLS_TUNING_FILE=gpurun_out/tune_c6.json timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench_c6_if5.log 2>&1 && \
MLS_TUNING_FILE=gpurun_out/tune_c6.json timeout -k 10 200 python bench.py --inflight 6 --steps 400 --warmup 40 > gpurun_out/bench_c6_if6.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench_c4_if5b.log 2>&1
