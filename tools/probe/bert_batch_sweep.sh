# BERT-base (config 3) throughput vs batch bucket: fused vs stock eager, 5 and 2 in flight.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/bert_sweep
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/bench_models.py bert --batches 16 32 64 128 --seqs 128 --steps 40 --inflight 5 > $OUT/if5.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/if5.jsonl
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 64 128 --seqs 128 --steps 40 --inflight 2 --backends fused > $OUT/if2.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/if2.jsonl
