# Halo kernel into the tuning table: numerics, per-layer re-score at c4, then bench A/B (shipped vs new table).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/halo_bench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halo_test.log 2>&1 && \
timeout -k 10 400 python tools/probe/halo_table_update.py > gpurun_out/halo_table.jsonl 2> gpurun_out/halo_table.err && \
timeout -k 10 300 python bench.py > gpurun_out/halo_bench.jsonl 2> gpurun_out/halo_bench.err && \
MLS_TUNING_FILE=gpurun_out/resnet50_gfx950_b32_halo.json timeout -k 10 300 python bench.py >> gpurun_out/halo_bench.jsonl 2>> gpurun_out/halo_bench.err && \
timeout -k 10 300 python bench.py >> gpurun_out/halo_bench.jsonl 2>> gpurun_out/halo_bench.err && \
MLS_TUNING_FILE=gpurun_out/resnet50_gfx950_b32_halo.json timeout -k 10 300 python bench.py >> gpurun_out/halo_bench.jsonl 2>> gpurun_out/halo_bench.err
