# re-tune the conv table for 4 co-running batches, then bench at inflight 5 with each table
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 900 python -u -m mlmicroservicetemplate_amd.ops.autotune --concurrency 4 --no-torch --out gpurun_out/tune_c4.json > gpurun_out/tune_c4.log 2>&1 && \
timeout -k 10 200 python bench.py --inflight 5 --steps 400 --warmup 40 > gpurun_out/bench_if5_shipped.log 2>&1 && \
MLS_TUNING_FILE=gpurun_out/tune_c4.json timeout -k 10 200 python bench.py --inflight 5 --steps 400 --warmup 40 > gpurun_out/bench_if5_c4.log 2>&1 && \
MLS_TUNING_FILE=gpurun_out/tune_c4.json timeout -k 10 200 python bench.py --inflight 8 --steps 400 --warmup 40 > gpurun_out/bench_if8_c4.log 2>&1 && \
MLS_SPLITK_INLAUNCH=0 MLS_TUNING_FILE=gpurun_out/tune_c4.json timeout -k 10 200 python bench.py --inflight 5 --steps 400 --warmup 40 > gpurun_out/bench_if5_c4_nosk.log 2>&1
