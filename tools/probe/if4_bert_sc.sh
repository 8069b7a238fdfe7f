# With slot-stream copies + pacing: 4 vs 5 in flight (one slot per hardware queue at 4); BERT A/B.
export TMPDIR=/tmp
CONFIGS="INFLIGHT=5
INFLIGHT=4" TAG=if4_s20 ROUNDS=3 STEPS=20 BENCH_ARGS="--warmup 5" bash tools/probe/proc_ab.sh || exit 1
CONFIGS="INFLIGHT=5
INFLIGHT=4" TAG=if4_s300 ROUNDS=1 STEPS=300 bash tools/probe/proc_ab.sh || exit 1
OUT=$GRAFT_REPO_ROOT/gpurun_out/bert_sc
mkdir -p $OUT
: > $OUT/ab.jsonl
for r in 1 2; do
  for v in 1 0; do
    MLS_SLOT_COPIES=$v timeout -k 10 200 python3 -u tools/bench_models.py bert --batches 32 128 --seqs 128 --steps 40 --inflight 5 --backends fused | sed "s/^{/{\"MLS_SLOT_COPIES\": $v, /" >> $OUT/ab.jsonl 2>> $OUT/err.log || exit 1
  done
done
cat $OUT/ab.jsonl | cut -c1-200
