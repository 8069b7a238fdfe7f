# Llama-3-8B TP=1 decode: bench (batch 1 / 8) + a rocprofv3 kernel trace of batch-1 decode steps.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama
mkdir -p $OUT
timeout -k 10 400 python3 tools/bench_models.py llama --batches 1 8 --steps 30 > $OUT/bench.jsonl 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench.jsonl
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/bench_models.py llama --batches 1 --steps 10 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
head -30 $OUT/kt/run_kernel_stats.csv | cut -c1-160
