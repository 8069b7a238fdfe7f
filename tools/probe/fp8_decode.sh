# FP8 (W8A8 e4m3) decode: numerics, then Llama-3-8B decode with MLS_DECODE_FP8 on / off (TP=1 and one
# emulated TP=8 rank).
OUT=$GRAFT_REPO_ROOT/gpurun_out/fp8
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_skinny_packed_gpu.py tests/test_kv_pages_gpu.py -k "fp8 or paged" > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for tp in 1 8; do
  for cfg in "MLS_DECODE_FP8=1" "MLS_DECODE_FP8=0"; do
    env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --emulate-tp $tp --batches 1 2 4 --steps 40 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    grep -v init_s $OUT/b.tmp | sed "s/^{/{\"cfg\": \"$cfg\", /" | tee -a $OUT/bench.jsonl
  done
done
