export TMPDIR=/tmp
OUT=gpurun_out/serve2
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 256 --prompt 128 --steps 10 > $OUT/decode256.jsonl 2> $OUT/decode256.err || { tail -20 $OUT/decode256.err; exit 1; }
cat $OUT/decode256.jsonl
S="tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64"
timeout -k 10 300 python3 -u $S > $OUT/serve_dev.jsonl 2> $OUT/serve_dev.err || { tail -20 $OUT/serve_dev.err; exit 1; }
cat $OUT/serve_dev.jsonl
MLS_SERVE_DEVICE_PICK=0 timeout -k 10 300 python3 -u $S > $OUT/serve_host.jsonl 2> $OUT/serve_host.err || { tail -20 $OUT/serve_host.err; exit 1; }
cat $OUT/serve_host.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gemm_tile_gpu.py tests/test_continuous_device_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; exit $rc
