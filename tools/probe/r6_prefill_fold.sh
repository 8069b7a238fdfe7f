# Round 6: Llama-3-8B TP=1 prefill with the residual add in the o / down epilogues (MLS_PREFILL_FOLD=1)
# vs the separate add + RMSNorm kernel; numerics tests with the fold on, then interleaved prefill A/B.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_prefill_fold}
mkdir -p $OUT
cd $R
MLS_PREFILL_FOLD=1 timeout -k 10 400 python3 -u -m pytest tests/test_models_gpu.py tests/test_continuous_device_gpu.py -x -q -k "llama or continuous" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
: > $OUT/llama.jsonl
for i in 1 2; do
  for v in 0 1; do
    MLS_PREFILL_FOLD=$v timeout -k 10 400 python3 tools/bench_models.py llama --batches 1 8 2>> $OUT/err \
      | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['prefill_fold']=$v; print(json.dumps(d))" >> $OUT/llama.jsonl || exit 1
  done
done
grep prefill_tok $OUT/llama.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l); print(d['prefill_fold'], d['batch'], d['prefill_tok_s'], d['decode_ms_per_step'])
"
