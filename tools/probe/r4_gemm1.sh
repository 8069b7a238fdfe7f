export TMPDIR=/tmp
OUT=gpurun_out/gemm1
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 1 8 --prompt 512 --steps 10 > $OUT/llama_native.jsonl 2> $OUT/llama_native.err || { tail -20 $OUT/llama_native.err; exit 1; }
cat $OUT/llama_native.jsonl
MLS_GEMM_IMPL=blas timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 1 8 --prompt 512 --steps 10 > $OUT/llama_blas.jsonl 2> $OUT/llama_blas.err || { tail -20 $OUT/llama_blas.err; exit 1; }
cat $OUT/llama_blas.jsonl
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/bert_native.jsonl 2> $OUT/bert_native.err || { tail -20 $OUT/bert_native.err; exit 1; }
cat $OUT/bert_native.jsonl
MLS_GEMM_IMPL=blas timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/bert_blas.jsonl 2> $OUT/bert_blas.err || { tail -20 $OUT/bert_blas.err; exit 1; }
cat $OUT/bert_blas.jsonl
timeout -k 10 400 python3 -u tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64 > $OUT/serve256.jsonl 2> $OUT/serve256.err || { tail -20 $OUT/serve256.err; exit 1; }
cat $OUT/serve256.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_llama8 -- python3 tools/bench_models.py llama --batches 8 --prompt 512 --steps 2 > $OUT/prof_llama8.log 2>&1 || { tail -20 $OUT/prof_llama8.log; exit 1; }
python3 tools/kernel_summary.py $OUT/prof_llama8 --top 30 > $OUT/prof_llama8_summary.txt 2>&1; head -40 $OUT/prof_llama8_summary.txt
