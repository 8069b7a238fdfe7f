# 8-phase (cfg 23) with k-half-outer MFMA order vs cfg 15, with / without DMA
export TMPDIR=/tmp
OUT=gpurun_out/r58pb
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_8p_gpu.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python3 -u tools/gemm_tile_probe.py --shapes sq8k bert128_ffn1 bert128_ffn2 bert128_qkv llama_o --cfgs 15 23 --conc 1 4 --ablate 1 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r58pb/probe.jsonl'):
    d=json.loads(l)
    if d.get('impl','').startswith('tile'): print(d['shape'], d['impl'], 'conc', d['conc'], d['us'])
PY
