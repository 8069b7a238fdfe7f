export TMPDIR=/tmp
OUT=gpurun_out/serve3
mkdir -p $OUT
timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 1 8 --prompt 512 --steps 10 > $OUT/llama.jsonl 2> $OUT/llama.err || { tail -20 $OUT/llama.err; exit 1; }
cat $OUT/llama.jsonl
S="tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64"
timeout -k 10 300 python3 -u $S > $OUT/serve_dev.jsonl 2> $OUT/serve_dev.err || { tail -20 $OUT/serve_dev.err; exit 1; }
cat $OUT/serve_dev.jsonl
timeout -k 10 300 python3 -u $S > $OUT/serve_dev2.jsonl 2>> $OUT/serve_dev.err || { tail -20 $OUT/serve_dev.err; exit 1; }
cat $OUT/serve_dev2.jsonl
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_e2e_gpu.py tests/test_continuous_device_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -3 $OUT/pytest.log; exit $rc
