# Llama-3-8B TP=1 decode / prefill and continuous-batching serving with the round-3 tree.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama3
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/bench_models.py llama --batches 1 8 32 128 --steps 20 > $OUT/decode.jsonl 2> $OUT/decode.err || { tail -20 $OUT/decode.err; exit 1; }
cat $OUT/decode.jsonl | cut -c1-250
timeout -k 10 500 python3 -u tools/bench_models.py llama-serve --batches 128 --requests 512 --new 64 > $OUT/serve.jsonl 2> $OUT/serve.err || { tail -20 $OUT/serve.err; exit 1; }
cat $OUT/serve.jsonl | cut -c1-300
