# Decode attention: numerics, then the Llama-3-8B TP=1 decode bench (batch 1 / 8 / 32).
OUT=$GRAFT_REPO_ROOT/gpurun_out/dattn
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_llama_tp_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
timeout -k 10 300 python3 tools/bench_models.py llama --batches 1 8 32 --steps 30 > $OUT/bench.jsonl 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
cat $OUT/bench.jsonl
