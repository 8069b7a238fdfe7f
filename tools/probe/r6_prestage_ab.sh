# Round 6: engine GPU tests, then interleaved bench arms: default (stage after the slot frees) vs
# MLS_BENCH_PRESTAGE=1 (next batch staged while the slots are busy, pulled by the graph straight from
# its pinned buffer through the slot's address cell -- no host memcpy into the slot buffer).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r6_prestage
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests/test_engine_gpu.py tests/test_gelu_epilogue_gpu.py tests/test_head_gpu.py tests/test_llama_tp_gpu.py -x -q -s --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
: > $OUT/bench.jsonl
for i in 1 2 3; do
  for arm in 0 1; do
    MLS_BENCH_PRESTAGE=$arm timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --measure-eager 0 > $OUT/b.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); d['arm']='prestage$arm'; print(json.dumps(d))" >> $OUT/bench.jsonl
  done
done
for arm in 0 1; do
  MLS_BENCH_PRESTAGE=$arm timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 --measure-eager 0 > $OUT/b.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open('$OUT/b.json')); d['arm']='prestage$arm'; print(json.dumps(d))" >> $OUT/bench.jsonl
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    d=json.loads(l); print(d['arm'], d['steps'], d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])
"
