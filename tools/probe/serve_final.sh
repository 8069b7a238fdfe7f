# Continuous-batching serving at 128 / 256 slots with the shipped tables.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/serve_final
mkdir -p $OUT
: > $OUT/serve.jsonl
for B in 128 256; do
  P=$((B * 3 + 1))
  timeout -k 10 400 python3 tools/bench_models.py llama-serve --batches $B --requests $((B * 4)) --prompt 128 --new 64 --kv-pages $P > $OUT/s.tmp 2> $OUT/s.err || { tail -20 $OUT/s.err; exit 1; }
  cat $OUT/s.tmp | tee -a $OUT/serve.jsonl
done
