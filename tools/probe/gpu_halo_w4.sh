# Halo variant 2 (64 channels x 4 waves): numerics, per-shape timing, per-layer re-score, bench A/B.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/halo_bench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halo_test.log 2>&1 && \
timeout -k 10 300 python tools/probe/halo_probe.py > gpurun_out/halo_w4_probe.jsonl 2>/dev/null && \
timeout -k 10 400 python tools/probe/halo_table_update.py > gpurun_out/halo_table.jsonl 2> gpurun_out/halo_table.err && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_bench.jsonl 2>/dev/null && \
MLS_TUNING_FILE=gpurun_out/resnet50_gfx950_b32_halo.json timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_bench.jsonl 2>/dev/null && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_bench.jsonl 2>/dev/null && \
MLS_TUNING_FILE=gpurun_out/resnet50_gfx950_b32_halo.json timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_bench.jsonl 2>/dev/null
