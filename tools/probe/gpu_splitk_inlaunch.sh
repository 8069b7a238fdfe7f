# A/B of the in-launch split-K reduction + correctness tests + a re-tune under 2-way concurrency
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_ops_gpu.py tests/test_models_gpu.py tests/test_engine_gpu.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t_splitk.log 2>&1 && \
MLS_SPLITK_INLAUNCH=0 timeout -k 10 200 python bench.py > gpurun_out/bench_off.log 2>&1 && \
timeout -k 10 200 python bench.py > gpurun_out/bench_on.log 2>&1 && \
timeout -k 10 600 python -u -m mlmicroservicetemplate_amd.ops.autotune --concurrency 2 --no-torch --out gpurun_out/tune_c2.json > gpurun_out/tune_c2.log 2>&1 && \
MLS_TUNING_FILE=gpurun_out/tune_c2.json timeout -k 10 200 python bench.py > gpurun_out/bench_on_retuned.log 2>&1
