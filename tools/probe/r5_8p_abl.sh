# 8-phase (cfg 23) vs cfg 15 with the DMA / store ablations: what bounds each main loop
export TMPDIR=/tmp
OUT=gpurun_out/r58pabl
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/gemm_tile_probe.py --shapes sq8k bert128_ffn1 bert128_ffn2 llama_o --cfgs 15 23 --conc 1 --ablate 1 2 3 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r58pabl/probe.jsonl'):
    d=json.loads(l)
    if d.get('impl','').startswith('tile'): print(d['shape'], d['impl'], 'ablate', d.get('ablate'), d['us'])
PY
