export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5llama2
mkdir -p $OUT
for r in 1 2; do
timeout -k 10 500 python3 -u tools/bench_models.py llama --batches 1 8 --steps 10 --prompt 512 > $OUT/prefill_$r.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
grep prefill_tok $OUT/prefill_$r.jsonl | cut -c1-200
done
