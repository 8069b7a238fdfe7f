export TMPDIR=/tmp
OUT=gpurun_out/dec256
mkdir -p $OUT
timeout -k 10 500 python3 -u tools/gemm_tile_probe.py --shapes dec256_qkv dec256_o dec256_gateup dec256_down dec256_lm --cfgs 1 2 3 4 5 15 16 --splitk 1 2 4 8 --conc 1 > $OUT/tile.jsonl 2> $OUT/tile.err || { tail -20 $OUT/tile.err; exit 1; }
timeout -k 10 500 python3 -u tools/gemm_probe.py --shapes dec256_qkv dec256_o dec256_down dec256_lm m256_gateup --splitk 1 2 4 8 > $OUT/conv.jsonl 2> $OUT/conv.err || { tail -20 $OUT/conv.err; exit 1; }
python3 - <<'PY'
import json
for f in ["tile", "conv"]:
    rows = [json.loads(l) for l in open(f"gpurun_out/dec256/{f}.jsonl") if '"us"' in l]
    for s in sorted({r["shape"] for r in rows}):
        rs = sorted([r for r in rows if r["shape"] == s], key=lambda r: r["us"])[:5]
        print(f, s, [(r["impl"], r.get("splitk"), r["us"]) for r in rs])
PY
