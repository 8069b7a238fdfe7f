export TMPDIR=/tmp
OUT=gpurun_out/pfg
mkdir -p $OUT
timeout -k 10 600 python3 -u tools/gemm_tile_probe.py --shapes llama_qkv llama_o llama_gateup llama_down llama32k_qkv llama32k_o llama32k_gateup llama32k_down --cfgs 1 15 --conc 1 --iters 5 > $OUT/tile.jsonl 2> $OUT/tile.err || { tail -20 $OUT/tile.err; exit 1; }
grep -v error $OUT/tile.jsonl | python3 -c "
import sys,json
for l in sys.stdin:
    d=json.loads(l)
    if 'us' in d: print(d['shape'], d['impl'], d['us'], d['tflops'], d['rel_err'])
"
