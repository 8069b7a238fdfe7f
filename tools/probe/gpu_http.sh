set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_service_gpu.py -x -v --timeout 300 --timeout-method thread -k "native" > gpurun_out/native_gpu_test.log 2>&1 && \
timeout -k 10 300 python -u tools/http_bench.py --model resnet50 --frontend native --io-threads 4 --client-threads 4 --conns 64 256 --duration 8 --warmup 2 > gpurun_out/http_native.jsonl 2> gpurun_out/http_native.err && \
timeout -k 10 300 python -u tools/http_bench.py --model resnet50 --frontend native --io-threads 6 --client-threads 6 --conns 256 --duration 8 --warmup 2 >> gpurun_out/http_native.jsonl 2>> gpurun_out/http_native.err
