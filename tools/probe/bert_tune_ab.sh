# A/B of the shipped TunableOp table (now with the BERT 64 / 128-bucket entries) vs the previous one.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/bert_tune
mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2; do
  timeout -k 10 200 python3 -u tools/bench_models.py bert --batches 32 64 128 --seqs 128 --steps 40 --inflight 5 --backends fused | sed 's/^{/{"table": "new", /' >> $OUT/ab.jsonl 2>> $OUT/err.log || exit 1
  MLS_BLAS_TUNING_FILE=$GRAFT_REPO_ROOT/tools/probe/alt_tables/tunableop_before_bert_b128.csv timeout -k 10 200 python3 -u tools/bench_models.py bert --batches 32 64 128 --seqs 128 --steps 40 --inflight 5 --backends fused | sed 's/^{/{"table": "old", /' >> $OUT/ab.jsonl 2>> $OUT/err.log || exit 1
done
cat $OUT/ab.jsonl
timeout -k 10 300 python3 -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k bert 2>&1 | tail -2
