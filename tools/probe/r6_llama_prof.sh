# Round 6: Llama-3-8B TP=1 B=8 x 512 prefill kernel summaries, native routes vs the hipBLASLt arm.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6_llama_prof
mkdir -p $OUT
cd $R
for arm in native blas; do
  e=""; [ $arm = blas ] && e="MLS_GEMM_IMPL=blas"
  env $e true
  if [ $arm = blas ]; then export MLS_GEMM_IMPL=blas; else unset MLS_GEMM_IMPL; fi
  timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/$arm -o run -- python3 -u tools/bench_models.py llama --batches 8 --steps 2 --prompt 512 > $OUT/$arm.jsonl 2> $OUT/$arm.err || { tail -20 $OUT/$arm.err; exit 1; }
  f=$(find $OUT/$arm -name "*kernel_trace.csv" | head -1)
  python3 tools/kernel_summary.py "$f" --top 25 > $OUT/$arm.summary.txt || exit 1
  rm -f "$f"
done
unset MLS_GEMM_IMPL
head -30 $OUT/native.summary.txt; head -30 $OUT/blas.summary.txt
