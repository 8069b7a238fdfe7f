# (cfg 24 = gemm_ring8_kernel was measured slower than cfg 15 / 23 and removed from gemm_tile.hip; kept as the record)
# cfg 24 (8-phase over a 10-slot half-tile ring: 7-8 phases of DMA lead) vs cfg 23 / 15: bitwise
# tests, then c1 / c4 timings with and without the DMA
export TMPDIR=/tmp
OUT=gpurun_out/r5ring8
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gemm_8p_gpu.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -1 $OUT/tests.log
timeout -k 10 600 python3 -u tools/gemm_tile_probe.py --shapes sq8k bert128_ffn1 bert128_ffn2 bert128_qkv llama_o llama_qkv --cfgs 15 23 24 --conc 1 4 --ablate 1 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r5ring8/probe.jsonl'):
    d=json.loads(l)
    if d.get('impl','').startswith('tile') or d.get('impl')=='hipblaslt': print(d['shape'], d['impl'], 'conc', d['conc'], d['us'])
PY
