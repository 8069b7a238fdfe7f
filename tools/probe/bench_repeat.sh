# Driver-like repeated runs: a GPU test file first, then bench.py --steps 20 --warmup 5 x4 and 300 x1.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/bench_repeat
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_engine_gpu.py tests/test_ops_gpu.py -x -q --timeout 200 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -20 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
: > $OUT/bench.jsonl
for i in 1 2 3 4; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $OUT/bench.jsonl 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 300 --warmup 20 >> $OUT/bench.jsonl 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    d=json.loads(l); print(d['steps'], d['value'], d['p50_latency_ms'], d['host_submit_ms_per_step'])
"
