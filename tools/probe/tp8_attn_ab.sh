# One emulated TP = 8 rank of Llama-3-8B (collectives stubbed): VALU vs matrix-core decode attention.
OUT=$GRAFT_REPO_ROOT/gpurun_out/tp8_attn
mkdir -p $OUT
: > $OUT/bench.jsonl
for v in valu mfma; do
  MLS_DECODE_ATTN=$v timeout -k 10 300 python3 -u tools/bench_models.py llama --emulate-tp 8 --batches ${BATCHES:-1 8 32 128} --steps 30 \
    > $OUT/b.tmp 2> $OUT/b.err || { tail -5 $OUT/b.err; exit 1; }
  sed "s/^{/{\"attn\": \"$v\", /" $OUT/b.tmp >> $OUT/bench.jsonl
done
cat $OUT/bench.jsonl
