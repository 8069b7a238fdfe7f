# 8-phase 256x256 tile (cfg 23) vs the shipped fragment-pipelined tile (cfg 15): bitwise tests, then
# c1 / c4 timings on the BERT / Llama / square shapes
export TMPDIR=/tmp
OUT=gpurun_out/r58p
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gemm_8p_gpu.py > $OUT/tests.log 2>&1 || { tail -40 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
timeout -k 10 600 python3 -u tools/gemm_tile_probe.py --shapes bert128_qkv bert128_o bert128_ffn1 bert128_ffn2 bert32_qkv bert32_ffn1 llama_o llama_qkv llama_down sq8k --cfgs 15 23 --conc 1 4 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 - <<'PY'
import json
for l in open('gpurun_out/r58p/probe.jsonl'):
    d=json.loads(l)
    print({k: d[k] for k in d if k in ('shape','impl','conc','us','tflops','rel_err','cfg')})
PY
