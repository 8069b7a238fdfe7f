# Native prefill index kernels: unit tests, every Llama GPU test, then the 256-slot serving bench and prefill.
export TMPDIR=/tmp
OUT=gpurun_out/pidx
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_prefill_index_gpu.py tests/test_kv_pages_gpu.py tests/test_continuous_device_gpu.py tests/test_e2e_gpu.py tests/test_llama_tp_gpu.py tests/test_models_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
S="tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64"
timeout -k 10 300 python3 -u $S > $OUT/serve1.jsonl 2> $OUT/serve.err || { tail -20 $OUT/serve.err; exit 1; }
tail -1 $OUT/serve1.jsonl
timeout -k 10 300 python3 -u $S > $OUT/serve2.jsonl 2>> $OUT/serve.err || { tail -20 $OUT/serve.err; exit 1; }
tail -1 $OUT/serve2.jsonl
timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 1 8 --prompt 512 --steps 10 > $OUT/llama.jsonl 2> $OUT/llama.err || { tail -20 $OUT/llama.err; exit 1; }
cat $OUT/llama.jsonl
