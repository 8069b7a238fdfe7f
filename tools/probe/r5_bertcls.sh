# BERT last layer on the [CLS] rows only (K/V projection of every token, Q + 1-query attention on [CLS])
# vs the full QKV + attention; small-M GEMM plans for the [CLS]-row projections
export TMPDIR=/tmp
OUT=gpurun_out/r5bertcls
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py tests/test_ln_fold_gpu.py -k "flash or bert" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
for r in 1 2; do
  for c in 1 0; do
    MLS_BERT_CLS_Q=$c timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/cls${c}_$r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    echo "cls_q=$c run $r"; cat $OUT/cls${c}_$r.jsonl
  done
done
timeout -k 10 400 python3 -u tools/gemm_probe.py --shapes bert32_o bert32_ffn1 bert32_ffn2 bert128_o bert128_ffn1 bert128_ffn2 --cfgs 0 2 3 6 11 15 16 17 24 25 26 --splitk 1 2 4 8 > $OUT/gemm.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
python3 - <<'PY'
import json
rs=[json.loads(l) for l in open('gpurun_out/r5bertcls/gemm.jsonl')]
for s in sorted({r['shape'] for r in rs}):
    x=sorted([r for r in rs if r['shape']==s], key=lambda r: r['us'])
    h=[r for r in x if r['impl']=='heuristic']
    print(s, 'best', [(r['impl'], r['splitk'], r['us']) for r in x[:3]], 'heuristic', [(r['splitk'], r['us']) for r in h][:1])
PY
