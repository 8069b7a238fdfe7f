# Paged KV cache cost: Llama-3-8B TP=1 decode (batch 1 / 8 / 32) and continuous-batching serving
# with per-slot caches vs a page pool (pages handed out in order / shuffled).
OUT=$GRAFT_REPO_ROOT/gpurun_out/paged
mkdir -p $OUT
for args in "--kv-pages 0" "--kv-pages 1100" "--kv-pages 1100 --shuffle-pages"; do
  timeout -k 10 300 python3 tools/bench_models.py llama --batches 1 8 32 --steps 30 $args > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  grep -v init_s $OUT/b.tmp | sed "s/^{/{\"args\": \"$args\", /" | tee -a $OUT/bench.jsonl
done
for args in "--kv-pages 0" "--kv-pages 400"; do
  timeout -k 10 300 python3 tools/bench_models.py llama-serve --batches 32 --requests 128 --prompt 128 --new 64 $args > $OUT/s.tmp 2> $OUT/s.err || { tail -20 $OUT/s.err; exit 1; }
  sed "s/^{/{\"args\": \"$args\", /" $OUT/s.tmp | tee -a $OUT/serve.jsonl
done
