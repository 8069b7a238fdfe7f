# Round 6: the 4-wave AGPR-accumulator tile GEMM (cfg 23) -- numerics vs cfg 15 / fp32, then the
# probe against cfg 15 and hipBLASLt on the BERT / Llama projection shapes.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r6_w4}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_gemm_tile_gpu.py -x -q -k "w4 or 23 or 24" --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
timeout -k 10 600 python3 tools/gemm_tile_probe.py --shapes ${SHAPES:-llama_o llama_down llama_qkv llama_gateup bert128_ffn1 bert128_qkv bert128_ffn2 sq8k} --cfgs 15 23 24 --conc ${CONC:-1} --iters 10 > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/probe.jsonl'):
    d=json.loads(l); print(d['shape'], d['impl'], d['conc'], d['us'], d['tflops'], d.get('rel_err'))"
