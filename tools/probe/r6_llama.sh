# Llama-3-8B TP=1 on the round-6 tree (every projection on native kernels): decode + prefill (B=1/8 x 512) and 256-slot continuous batching
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6llama
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/bench_models.py llama --batches 1 8 --steps 20 --prompt 512 > $OUT/decode_prefill.jsonl 2> $OUT/decode.err || { tail -20 $OUT/decode.err; exit 1; }
cut -c1-300 $OUT/decode_prefill.jsonl
timeout -k 10 600 python3 -u tools/bench_models.py llama-serve --batches 256 --requests 1024 --new 64 --prompt 128 > $OUT/serve.jsonl 2> $OUT/serve.err || { tail -20 $OUT/serve.err; exit 1; }
cut -c1-300 $OUT/serve.jsonl
# the same prefill with hipBLASLt for every plain projection (the A/B arm, MLS_GEMM_IMPL=blas)
MLS_GEMM_IMPL=blas timeout -k 10 500 python3 -u tools/bench_models.py llama --batches 1 8 --steps 10 --prompt 512 > $OUT/prefill_blas_arm.jsonl 2> $OUT/blas.err || { tail -20 $OUT/blas.err; exit 1; }
grep prefill_tok $OUT/prefill_blas_arm.jsonl | cut -c1-200
