# Halo kernel: register-staged chunk prefetch (default) vs LDS-DMA per chunk: numerics for both,
# per-layer timing, bench A/B.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/halo_rs.jsonl gpurun_out/halo_rs_bench.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halo_rs_test.log 2>&1 && \
MLS_HALO_RS=0 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo" >> gpurun_out/halo_rs_test.log 2>&1 && \
timeout -k 10 300 python tools/probe/halo_probe.py 2>/dev/null | sed 's/^{/{"rs": 1, /' >> gpurun_out/halo_rs.jsonl && \
MLS_HALO_RS=0 timeout -k 10 300 python tools/probe/halo_probe.py 2>/dev/null | sed 's/^{/{"rs": 0, /' >> gpurun_out/halo_rs.jsonl && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_rs_bench.jsonl 2>/dev/null && \
MLS_HALO_RS=0 timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_rs_bench.jsonl 2>/dev/null && \
timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_rs_bench.jsonl 2>/dev/null && \
MLS_HALO_RS=0 timeout -k 10 200 python bench.py --steps 400 --warmup 40 >> gpurun_out/halo_rs_bench.jsonl 2>/dev/null
