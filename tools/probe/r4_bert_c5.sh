export TMPDIR=/tmp
OUT=gpurun_out/bertc5
mkdir -p $OUT
timeout -k 10 900 python3 -u tools/gemm_tile_probe.py --shapes bert128_qkv bert128_o bert128_ffn1 bert128_ffn2 bert32_qkv bert32_o bert32_ffn1 bert32_ffn2 --cfgs 1 2 5 15 16 21 22 --conc 5 --iters 10 > $OUT/tile.jsonl 2> $OUT/err.log || { tail -5 $OUT/err.log; exit 1; }
python3 -c "
import json
rows=[json.loads(l) for l in open('$OUT/tile.jsonl') if '\"us\"' in l]
for s in sorted({r['shape'] for r in rows}):
    rs=sorted([r for r in rows if r['shape']==s], key=lambda r:r['us'])[:4]
    print(s, [(r['impl'], r['us']) for r in rs])
"
