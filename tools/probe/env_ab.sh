# Llama-3-8B TP=1 decode A/B of one environment switch: VAR=NAME VALS="0 1" BATCHES="64 128".
OUT=$GRAFT_REPO_ROOT/gpurun_out/env_ab
mkdir -p $OUT
: > $OUT/bench.jsonl
for v in ${VALS:-0 1}; do
  env $VAR=$v timeout -k 10 300 python3 -u tools/bench_models.py llama --batches ${BATCHES:-64 128} --steps 20 \
    > $OUT/b.tmp 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  sed "s/^{/{\"$VAR\": \"$v\", /" $OUT/b.tmp >> $OUT/bench.jsonl
done
cat $OUT/bench.jsonl
