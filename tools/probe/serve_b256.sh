# Continuous-batching serving at 128 / 256 decode slots (paged KV, 3 pages per slot).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/serve256
mkdir -p $OUT
for B in 128 256; do
  P=$((B * 3 + 1))
  timeout -k 10 400 python3 tools/bench_models.py llama-serve --batches $B --requests $((B * 4)) --prompt 128 --new 64 --kv-pages $P > $OUT/s.tmp 2> $OUT/s.err || { tail -20 $OUT/s.err; exit 1; }
  cat $OUT/s.tmp | tee -a $OUT/serve.jsonl
done
timeout -k 10 300 python3 tools/bench_models.py llama --batches 128 256 --prompt 128 --steps 20 > $OUT/decode.jsonl 2>> $OUT/s.err || { tail -20 $OUT/s.err; exit 1; }
cat $OUT/decode.jsonl
