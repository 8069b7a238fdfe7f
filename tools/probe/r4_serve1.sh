export TMPDIR=/tmp
OUT=gpurun_out/serve1
mkdir -p $OUT
S="tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64"
MLS_SERVE_DEVICE_PICK=0 timeout -k 10 300 python3 -u $S > $OUT/serve_host.jsonl 2> $OUT/serve_host.err || { tail -20 $OUT/serve_host.err; exit 1; }
cat $OUT/serve_host.jsonl
MLS_GEMM_IMPL=blas timeout -k 10 300 python3 -u $S > $OUT/serve_dev_blas.jsonl 2> $OUT/serve_dev_blas.err || { tail -20 $OUT/serve_dev_blas.err; exit 1; }
cat $OUT/serve_dev_blas.jsonl
timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 128 256 --prompt 128 --steps 10 > $OUT/decode_native.jsonl 2> $OUT/decode_native.err || { tail -20 $OUT/decode_native.err; exit 1; }
cat $OUT/decode_native.jsonl
MLS_GEMM_IMPL=blas timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 128 256 --prompt 128 --steps 10 > $OUT/decode_blas.jsonl 2> $OUT/decode_blas.err || { tail -20 $OUT/decode_blas.err; exit 1; }
cat $OUT/decode_blas.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serve -- python3 tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 256 --prompt 128 --new 64 > $OUT/prof_serve.log 2>&1 || { tail -20 $OUT/prof_serve.log; exit 1; }
python3 tools/kernel_summary.py $OUT/prof_serve --top 40 > $OUT/prof_serve_summary.txt 2>&1; head -45 $OUT/prof_serve_summary.txt
