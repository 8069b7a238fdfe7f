# Packed decode GEMMs up to 32 rows: numerics, then Llama-3-8B TP=1 decode at batch 1..32, packed on / off.
OUT=$GRAFT_REPO_ROOT/gpurun_out/packed32
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_skinny_packed_gpu.py tests/test_llama_tp_gpu.py > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for cfg in "MLS_PACKED_DECODE=1" "MLS_PACKED_VARIANT=10" "MLS_PACKED_DECODE=0"; do
  env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --batches 16 24 32 --steps 30 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  sed "s/^{/{\"cfg\": \"$cfg\", /" $OUT/b.tmp | tee -a $OUT/bench.jsonl
done
