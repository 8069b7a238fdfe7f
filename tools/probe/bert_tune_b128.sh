# TunableOp search for BERT-base at the 64 / 128 buckets, then A/B of the merged table.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/bert_tune
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/tune_bert_blas.py --batches 64 128 --out $OUT/tuned.csv > $OUT/tune.log 2>&1 || { tail -30 $OUT/tune.log; exit 1; }
grep tuned $OUT/tune.log
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/bench_models.py bert --batches 64 128 --seqs 128 --steps 40 --inflight 5 --backends fused | sed 's/^{/{"table": "default", /' >> $OUT/ab.jsonl 2>> $OUT/err.log || exit 1
  MLS_BLAS_TUNING_FILE=$OUT/tuned.csv timeout -k 10 200 python3 -u tools/bench_models.py bert --batches 64 128 --seqs 128 --steps 40 --inflight 5 --backends fused | sed 's/^{/{"table": "tuned", /' >> $OUT/ab.jsonl 2>> $OUT/err.log || exit 1
done
cat $OUT/ab.jsonl
