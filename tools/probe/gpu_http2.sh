# Native front end end-to-end (ResNet-50, 150 KB multipart uploads) at 128 / 256 / 384 connections.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/http_bench.py --model resnet50 --frontend native --io-threads 4 --client-threads 4 --conns 128 256 --duration 8 --warmup 2 > gpurun_out/http_native2.jsonl 2> gpurun_out/http_native2.err && \
timeout -k 10 300 python -u tools/http_bench.py --model resnet50 --frontend native --io-threads 6 --client-threads 6 --conns 256 384 --duration 8 --warmup 2 >> gpurun_out/http_native2.jsonl 2>> gpurun_out/http_native2.err
