# TunableOp search for the Llama-3-8B TP=1 projections at 256 rows (256-slot serving), then A/B.
# (TunableOp appends the device ordinal to PYTORCH_TUNABLEOP_FILENAME: tuned.csv -> tuned0.csv)
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama_m256
mkdir -p $OUT
if [ ! -s $OUT/tuned0.csv ]; then
  PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=$OUT/tuned.csv timeout -k 10 600 python3 -u tools/tune_llama_blas.py --m 256 > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
fi
grep -v "^Validator" $OUT/tuned0.csv > $OUT/new_rows.csv
cp mlmicroservicetemplate_amd/ops/tuned/tunableop_gfx950.csv $OUT/merged.csv && cat $OUT/new_rows.csv >> $OUT/merged.csv
: > $OUT/ab.jsonl
for r in 1 2; do
  timeout -k 10 300 python3 tools/bench_models.py llama --batches 256 --prompt 128 --steps 20 2>>$OUT/err.log | grep decode | sed 's/^{/{"table": "shipped", /' >> $OUT/ab.jsonl || exit 1
  MLS_BLAS_TUNING_FILE=$OUT/merged.csv timeout -k 10 300 python3 tools/bench_models.py llama --batches 256 --prompt 128 --steps 20 2>>$OUT/err.log | grep decode | sed 's/^{/{"table": "m256", /' >> $OUT/ab.jsonl || exit 1
done
cat $OUT/ab.jsonl | cut -c1-220
