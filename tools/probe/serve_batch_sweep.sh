# Continuous-batching serving throughput vs decode slots (paged KV pool sized for the slots).
OUT=$GRAFT_REPO_ROOT/gpurun_out/serve
mkdir -p $OUT
for B in 32 64 128; do
  P=$((B * 3 + 1))
  timeout -k 10 300 python3 tools/bench_models.py llama-serve --batches $B --requests $((B * 4)) --prompt 128 --new 64 --kv-pages $P > $OUT/s.tmp 2> $OUT/s.err || { tail -20 $OUT/s.err; exit 1; }
  cat $OUT/s.tmp | tee -a $OUT/serve.jsonl
done
