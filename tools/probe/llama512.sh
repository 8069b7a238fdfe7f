export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama512
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/bench_models.py llama --batches 1 8 --steps 10 > $OUT/after.jsonl 2> $OUT/after.err || { tail -20 $OUT/after.err; exit 1; }
cat $OUT/after.jsonl | cut -c1-250
timeout -k 10 300 python3 -u -m pytest tests/test_e2e_gpu.py tests/test_gemm_tile_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
