# Llama-3-8B TP=1 decode: bench (batch 1 / 8) + a rocprofv3 kernel trace of decode steps at
# batch ${TRACE_BATCH:-1}, reduced to the last step's per-kernel breakdown.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama
B=${TRACE_BATCH:-1}
mkdir -p $OUT
if [ -z "$SKIP_BENCH" ]; then
  timeout -k 10 400 python3 tools/bench_models.py llama --batches 1 8 --steps 30 > $OUT/bench.jsonl 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.jsonl
fi
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_b$B -o run -- python3 tools/bench_models.py llama --batches $B --steps 10 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 tools/probe/decode_step_breakdown.py $OUT/kt_b$B/run_kernel_trace.csv | tee $OUT/breakdown_b$B.txt
