# o-projection with the split-KV combine in its prologue: numerics, then decode A/B (TP=1 and one
# emulated TP=8 rank, batch 1 / 4), MLS_FUSE_COMBINE on / off.
OUT=$GRAFT_REPO_ROOT/gpurun_out/fcomb
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_skinny_packed_gpu.py tests/test_llama_tp_gpu.py tests/test_kv_pages_gpu.py tests/test_models_gpu.py -k "combine or llama or paged or continuous or generate" > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for tp in 1 8; do
  for cfg in "MLS_FUSE_COMBINE=1" "MLS_FUSE_COMBINE=0"; do
    env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --emulate-tp $tp --batches 1 4 --steps 40 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    grep -v init_s $OUT/b.tmp | sed "s/^{/{\"cfg\": \"$cfg\", /" | tee -a $OUT/bench.jsonl
  done
done
