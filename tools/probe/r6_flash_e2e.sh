# Round 6: flash v2 tests + Llama-3-8B TP=1 prefill / decode with flash v1 vs v2 (interleaved).
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_flash_e2e}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_ops_gpu.py tests/test_models_gpu.py -x -q -k "flash or llama or attention" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
: > $OUT/llama.jsonl
for i in 1 2; do
  for v in 1 2; do
    MLS_FLASH_V=$v timeout -k 10 400 python3 tools/bench_models.py llama --batches 1 8 2>> $OUT/err \
      | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['flash_v']=$v; print(json.dumps(d))" >> $OUT/llama.jsonl || exit 1
  done
done
grep prefill $OUT/llama.jsonl
