# Round 6: medium-M GEMM route (MLS_MGEMM) -- tests, then Llama-3-8B TP=1 decode at 64/128/256 rows
# and 256-slot continuous batching, interleaved MLS_MGEMM=0 / 1.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_mgemm_e2e}
mkdir -p $OUT
cd $R
timeout -k 10 600 python3 -u -m pytest tests/test_mgemm_gpu.py tests/test_models_gpu.py tests/test_continuous_device_gpu.py -x -q -k "mgemm or llama or continuous" --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
: > $OUT/llama.jsonl
for i in ${ROUNDS_SEQ:-1 2}; do
  for v in 0 1; do
    MLS_MGEMM=$v timeout -k 10 400 python3 tools/bench_models.py llama --batches ${BATCHES:-64 128 256} --prompt 128 2>> $OUT/err \
      | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['mgemm']=$v; print(json.dumps(d))" >> $OUT/llama.jsonl || exit 1
    MLS_MGEMM=$v timeout -k 10 400 python3 tools/bench_models.py llama-serve --batches ${SERVE:-256} --requests $((4 * ${SERVE:-256})) --prompt 128 --new 64 2>> $OUT/err \
      | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['mgemm']=$v; print(json.dumps(d))" >> $OUT/llama.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/llama.jsonl'):
    d=json.loads(l)
    if 'decode_ms_per_step' in d or 'tokens_per_s' in d: print(d.get('mgemm'), d.get('batch', d.get('max_batch')), d.get('decode_ms_per_step'), d.get('prefill_tok_s'), d.get('tokens_per_s'))"
