# Round 6: flash v2 for BERT's 8-wave D = 64 blocks: tests, then the BERT engine (B = 32 / 64 / 128,
# 200 ms warm floor) with MLS_FLASH_V = 1 / 2 interleaved.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_flash_bert}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_ops_gpu.py tests/test_models_gpu.py tests/test_ln_fold_gpu.py -x -q -k "flash or bert or attention or fold" --timeout 200 --timeout-method thread > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
: > $OUT/bert.jsonl
for i in 1 2; do
  for v in 1 2; do
    MLS_FLASH_V=$v timeout -k 10 300 python3 tools/bench_models.py bert --backends fused --batches 32 64 128 2>> $OUT/err \
      | python3 -c "import sys,json
for l in sys.stdin:
    d=json.loads(l); d['flash_v']=$v; print(json.dumps(d))" >> $OUT/bert.jsonl || exit 1
  done
done
python3 -c "
import json
for l in open('$OUT/bert.jsonl'):
    d=json.loads(l)
    if 'seq_per_s' in d: print(d['flash_v'], d['batch'], d['seq_per_s'])
"
