# Llama-3-8B TP=1 decode at batch 32 / 64 / 128 with and without the TunableOp table
# (MLS_BLAS_TUNING=0 leaves hipBLASLt on its default heuristic).
OUT=$GRAFT_REPO_ROOT/gpurun_out/blas_ab
mkdir -p $OUT
: > $OUT/bench.jsonl
for t in 0 1; do
  MLS_BLAS_TUNING=$t timeout -k 10 300 python3 -u tools/bench_models.py llama --batches ${BATCHES:-32 64 128} --steps 20 \
    > $OUT/b.tmp 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  sed "s/^{/{\"blas_tuning\": $t, /" $OUT/b.tmp >> $OUT/bench.jsonl
done
cat $OUT/bench.jsonl
