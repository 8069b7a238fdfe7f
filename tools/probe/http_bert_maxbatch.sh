# BERT over HTTP (native front end, C++ tokenizer): batch cap 32 vs 128 (dynamic batcher buckets).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/http_bert_mb
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --conns 256 --duration 6 --warmup 2 --ready-timeout 200 | sed 's/^{/{"MAX_BATCH": 32, /' > $OUT/r.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
MAX_BATCH=128 timeout -k 10 300 python3 -u tools/http_bench.py --model bert --frontend native --text --io-threads 4 --client-threads 4 --conns 256 512 --duration 6 --warmup 2 --ready-timeout 200 | sed 's/^{/{"MAX_BATCH": 128, /' >> $OUT/r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/r.jsonl
