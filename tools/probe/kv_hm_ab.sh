# Head-major KV caches: numerics, then Llama-3-8B TP=1 decode at batch 1 / 8 / 32 / 128 with
# MLS_KV_HEAD_MAJOR on / off.
OUT=$GRAFT_REPO_ROOT/gpurun_out/kvhm
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_kv_pages_gpu.py tests/test_transformer_ops_gpu.py tests/test_llama_tp_gpu.py tests/test_models_gpu.py -k "paged or head_major or decode or rope or llama or continuous or generate" > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for cfg in ${CFGS:-"MLS_KV_HEAD_MAJOR=1" "MLS_KV_HEAD_MAJOR=0"}; do
  env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --batches 1 8 32 128 --steps 20 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  grep -v init_s $OUT/b.tmp | sed "s/^{/{\"cfg\": \"$cfg\", /" | tee -a $OUT/bench.jsonl
done
