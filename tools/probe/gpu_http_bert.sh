# Config 3 end to end: BERT-base text classifier over real HTTP (100-word texts, multipart field `text`),
# dynamic batching through the native C++ front end (tokenised straight into packed engine rows).
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_service_gpu.py -x -v --timeout 300 --timeout-method thread -k "bert" > gpurun_out/bert_native_test.log 2>&1 && \
timeout -k 10 300 python -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --conns 64 256 --duration 8 --warmup 2 --ready-timeout 200 > gpurun_out/http_bert.jsonl 2> gpurun_out/http_bert.err && \
timeout -k 10 300 python -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --decode-workers 4 --conns 512 --duration 8 --warmup 2 --ready-timeout 200 >> gpurun_out/http_bert.jsonl 2>> gpurun_out/http_bert.err
