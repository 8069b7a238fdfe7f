# Round 6: BERT (B=32/64/128) and Llama-3-8B TP=1 prefill / decode with and without the 200 ms
# warm floor (tools/bench_models.py --warm-ms), interleaved.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r6_models_warm}
mkdir -p $OUT
: > $OUT/bert.jsonl
for i in 1 2; do
  for w in 0 200; do
    timeout -k 10 240 python3 tools/bench_models.py bert --backends fused --batches 32 64 128 --warm-ms $w 2>> $OUT/err \
      | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['warm_ms']=$w; print(json.dumps(d))" >> $OUT/bert.jsonl || exit 1
  done
done
: > $OUT/llama.jsonl
for w in 0 200; do
  timeout -k 10 400 python3 tools/bench_models.py llama --batches 1 8 --warm-ms $w 2>> $OUT/err \
    | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['warm_ms']=$w; print(json.dumps(d))" >> $OUT/llama.jsonl || exit 1
done
cat $OUT/bert.jsonl $OUT/llama.jsonl
