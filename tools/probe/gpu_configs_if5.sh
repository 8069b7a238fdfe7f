# configs 2/3 at 5 batches in flight: eager baseline (same engine), BERT, native HTTP
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --backend eager --inflight 5 --steps 100 --warmup 10 > gpurun_out/bench_eager_if5.log 2>&1 && \
timeout -k 10 300 python bench.py --backend eager --inflight 3 --steps 100 --warmup 10 > gpurun_out/bench_eager_if3.log 2>&1 && \
timeout -k 10 300 python -u tools/bench_models.py bert --batches 32 --inflight 5 > gpurun_out/bert_if5.jsonl 2> gpurun_out/bert_if5.err && \
timeout -k 10 300 python -u tools/bench_models.py bert --batches 32 --inflight 3 > gpurun_out/bert_if3.jsonl 2> gpurun_out/bert_if3.err && \
timeout -k 10 300 python -u tools/http_bench.py --model resnet50 --frontend native --io-threads 4 --client-threads 4 --conns 128 256 512 --duration 8 --warmup 2 > gpurun_out/http_native_if5.jsonl 2> gpurun_out/http_native_if5.err
