# Continuous batching after vectorising the per-iteration host work: 128 / 256 slots + GPU test.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/serve_host
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_models_gpu.py tests/test_kv_pages_gpu.py -x -q --timeout 200 --timeout-method thread -k "continuous or paged" > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
: > $OUT/serve.jsonl
for B in 128 256; do
  P=$((B * 3 + 1))
  timeout -k 10 400 python3 tools/bench_models.py llama-serve --batches $B --requests $((B * 4)) --prompt 128 --new 64 --kv-pages $P > $OUT/s.tmp 2> $OUT/s.err || { tail -20 $OUT/s.err; exit 1; }
  cat $OUT/s.tmp | tee -a $OUT/serve.jsonl
done
