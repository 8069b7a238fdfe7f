set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest tests/test_ops_gpu.py -x -q --timeout 120 --timeout-method thread -k "stem" > gpurun_out/stem_test.log 2>&1 && \
timeout -k 10 200 python tools/probe/stem_pool_probe.py > gpurun_out/stem_probe.jsonl 2> gpurun_out/stem_probe.err
