# fused stem kernel: numerics vs the 3-kernel path, timing, then the flagship bench both ways
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem" > gpurun_out/stem_test.log 2>&1 && \
timeout -k 10 200 python tools/probe/stem_pool_probe.py > gpurun_out/stem_probe.jsonl 2> gpurun_out/stem_probe.err && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench_stemfused.log 2>&1 && \
MLS_FUSED_STEM=0 timeout -k 10 200 python bench.py --steps 400 --warmup 40 > gpurun_out/bench_stem3.log 2>&1 && \
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke2.log 2>&1
