# TunableOp search for the Llama-3-8B prefill projections at 16k / 32k rows (128 / 256 admitted
# 128-token prompts), then prefill + serving A/B against the shipped table.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama_prefill_tune
mkdir -p $OUT
PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tuned.csv timeout -k 10 800 python3 -u tools/tune_llama_blas.py --m 16384 32768 --shapes qkv o gate_up down > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
grep tuned $OUT/tune.log
grep -v "^Validator" $OUT/tuned0.csv > $OUT/new_rows.csv
cat $OUT/new_rows.csv
cp mlmicroservicetemplate_amd/ops/tuned/tunableop_gfx950.csv $OUT/merged.csv && cat $OUT/new_rows.csv >> $OUT/merged.csv
: > $OUT/ab.jsonl
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_models.py llama --batches 128 256 --prompt 128 --steps 5 2>>$OUT/err.log | grep prefill | sed 's/^{/{"table": "shipped", /' >> $OUT/ab.jsonl || exit 1
  MLS_BLAS_TUNING_FILE=$OUT/merged.csv timeout -k 10 300 python3 tools/bench_models.py llama --batches 128 256 --prompt 128 --steps 5 2>>$OUT/err.log | grep prefill | sed 's/^{/{"table": "prefill", /' >> $OUT/ab.jsonl || exit 1
done
cat $OUT/ab.jsonl | cut -c1-220
