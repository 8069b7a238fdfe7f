# Llama-3-8B (TP=1) native tile GEMMs vs the hipBLASLt arm: prefill + decode (bench_models llama)
# and continuous-batching serving at 256 slots.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-llama_ab}
mkdir -p $OUT
for impl in native blas; do
  MLS_GEMM_IMPL=$impl timeout -k 10 300 python3 tools/bench_models.py llama --batches 1 8 --steps 20 > $OUT/llama_$impl.jsonl 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  sed "s/^/$impl /" $OUT/llama_$impl.jsonl
  MLS_GEMM_IMPL=$impl timeout -k 10 400 python3 tools/bench_models.py llama-serve --batches 256 --requests 1024 --prompt 128 --new 64 --kv-pages 769 > $OUT/serve_$impl.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  sed "s/^/$impl /" $OUT/serve_$impl.jsonl
done
