# Round 6: Llama-3-8B TP=1 decode (BATCHES rows, 128-token prompts) and continuous serving (SERVE
# slots) interleaved over ARMS="name:ENV=V,... name2:..." (ROUNDS_SEQ rounds); optional TESTS first.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_llama_ab}
mkdir -p $OUT
cd $R
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python3 -u -m pytest $TESTS -x -q --timeout 300 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
  tail -2 $OUT/tests.log
fi
: > $OUT/llama.jsonl
tagged() { python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['arm']='$1'; print(json.dumps(d))"; }
for i in ${ROUNDS_SEQ:-1 2}; do
  for arm in $ARMS; do
    name=${arm%%:*}; envs=${arm#*:}; e=""; [ "$envs" != "$arm" ] && e=$(echo "$envs" | tr ',' ' ')
    env $e timeout -k 10 400 python3 tools/bench_models.py llama --batches ${BATCHES:-32 64 128 256} --prompt 128 2>> $OUT/err | tagged $name >> $OUT/llama.jsonl || exit 1
    if [ -n "${SERVE:-256}" ] && [ "${SERVE:-256}" != "0" ]; then
      env $e timeout -k 10 400 python3 tools/bench_models.py llama-serve --batches ${SERVE:-256} --requests $((4 * ${SERVE:-256})) --prompt 128 --new 64 2>> $OUT/err | tagged $name >> $OUT/llama.jsonl || exit 1
    fi
  done
done
python3 -c "
import json
for l in open('$OUT/llama.jsonl'):
    d=json.loads(l)
    if 'decode_ms_per_step' in d or 'tokens_per_s' in d: print(d['arm'], d.get('batch', d.get('max_batch')), d.get('decode_ms_per_step'), d.get('prefill_tok_s'), d.get('tokens_per_s'))"
