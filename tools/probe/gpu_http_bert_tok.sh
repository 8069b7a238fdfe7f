# bert over HTTP: Python decode threads vs the C++ I/O-thread tokenizer, with server-side mean batch
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --conns 64 256 --duration 6 --warmup 2 --ready-timeout 200 > gpurun_out/http_bert_tok.jsonl 2> gpurun_out/http_bert_tok.err && \
MLS_NATIVE_TOKENIZER=1 timeout -k 10 300 python -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --conns 64 256 --duration 6 --warmup 2 --ready-timeout 200 >> gpurun_out/http_bert_tok.jsonl 2>> gpurun_out/http_bert_tok.err && \
MLS_NATIVE_TOKENIZER=1 MAX_WAIT_US=500 timeout -k 10 300 python -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --conns 64 --duration 6 --warmup 2 --ready-timeout 200 >> gpurun_out/http_bert_tok.jsonl 2>> gpurun_out/http_bert_tok.err
