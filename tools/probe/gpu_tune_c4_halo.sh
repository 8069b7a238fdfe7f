# Full re-tune at 4-way concurrency with the halo candidates, then bench A/B (shipped vs new), 2 runs each.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/tune_halo_bench.jsonl
timeout -k 10 1000 python -u -m mlmicroservicetemplate_amd.ops.autotune --concurrency 4 --no-torch --out gpurun_out/tune_c4_halo.json > gpurun_out/tune_c4_halo.log 2>&1 && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/tune_halo_bench.jsonl 2> gpurun_out/tune_halo_bench.err && \
MLS_TUNING_FILE=gpurun_out/tune_c4_halo.json timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/tune_halo_bench.jsonl 2>> gpurun_out/tune_halo_bench.err && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/tune_halo_bench.jsonl 2>> gpurun_out/tune_halo_bench.err && \
MLS_TUNING_FILE=gpurun_out/tune_c4_halo.json timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/tune_halo_bench.jsonl 2>> gpurun_out/tune_halo_bench.err
