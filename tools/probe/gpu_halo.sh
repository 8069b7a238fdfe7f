# Halo 3x3 kernel: numerics first (stop on failure), then timing vs the implicit GEMM, for the
# single-stage (2 blocks / CU) and double-buffered variants.
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/halo_probe.jsonl
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -v --timeout 120 --timeout-method thread -k "halo" > gpurun_out/halo_test.log 2>&1 && \
MLS_HALO_STAGES=2 timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "halo" >> gpurun_out/halo_test.log 2>&1 && \
timeout -k 10 300 python tools/probe/halo_probe.py 2> gpurun_out/halo_probe.err | sed 's/^{/{"stages": 1, /' >> gpurun_out/halo_probe.jsonl && \
MLS_HALO_STAGES=2 timeout -k 10 300 python tools/probe/halo_probe.py 2>> gpurun_out/halo_probe.err | sed 's/^{/{"stages": 2, /' >> gpurun_out/halo_probe.jsonl
