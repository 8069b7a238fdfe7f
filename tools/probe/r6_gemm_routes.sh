# Round 6: every native kernel config on the nine shapes the tile table used to route to hipBLASLt
# (Llama-3-8B TP=1: 512-row QKV / O, the 256-row decode O / down / LM head, QKV / O / gate_up / down
# from 1024 rows), hipBLASLt timed alongside as the reference line.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_gemm_routes
mkdir -p $OUT
timeout -k 10 400 python3 -u tools/gemm_tile_probe.py --shapes llama512_qkv llama512_o dec256_o dec256_down dec256_lm --cfgs 1 2 4 5 15 16 21 22 --splitk 1 2 4 8 --conc 1 > $OUT/tile_small.jsonl 2> $OUT/tile_small.err || { tail -20 $OUT/tile_small.err; exit 1; }
timeout -k 10 300 python3 -u tools/gemm_probe.py --shapes dec256_o dec256_down dec256_lm --cfgs 0 1 2 3 4 5 6 7 8 9 10 11 12 --splitk 1 2 4 8 > $OUT/conv_small.jsonl 2> $OUT/conv_small.err || { tail -20 $OUT/conv_small.err; exit 1; }
timeout -k 10 500 python3 -u tools/gemm_tile_probe.py --shapes llama_qkv llama_o llama_gateup llama_down llama32k_qkv llama32k_o llama32k_down --cfgs 1 2 4 5 15 16 21 22 --splitk 1 --conc 1 --iters 5 > $OUT/tile_big.jsonl 2> $OUT/tile_big.err || { tail -20 $OUT/tile_big.err; exit 1; }
python3 - <<'PY'
import json, os
out = os.environ["GRAFT_REPO_ROOT"] + "/gpurun_out/r6_gemm_routes"
for f in ["tile_small", "conv_small", "tile_big"]:
    rows = [json.loads(l) for l in open(f"{out}/{f}.jsonl") if '"us"' in l]
    for s in sorted({r["shape"] for r in rows}):
        rs = [r for r in rows if r["shape"] == s]
        ref = [r for r in rs if r["impl"] in ("hipblaslt", "torch")]
        nat = sorted([r for r in rs if r["impl"] not in ("hipblaslt", "torch")], key=lambda r: r["us"])[:4]
        print(f, s, "lib", [r["us"] for r in ref], "native", [(r["impl"], r.get("splitk"), r["us"], r.get("rel_err")) for r in nat])
PY
