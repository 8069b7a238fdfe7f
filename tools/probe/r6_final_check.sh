# Round 6 final-tree check: full GPU suite, smoke, three driver-form benches, one 200-step bench.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_final_check}
mkdir -p $OUT
cd $R
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/suite.log 2>&1 || { tail -30 $OUT/suite.log; exit 1; }
tail -1 $OUT/suite.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
: > $OUT/s20.jsonl
for r in 1 2 3; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $OUT/s20.jsonl 2>> $OUT/s20.err || { tail -20 $OUT/s20.err; exit 1; }
done
timeout -k 10 400 python3 bench.py > $OUT/default.json 2> $OUT/default.err || { tail -20 $OUT/default.err; exit 1; }
python3 -c "
import json
for l in open('$OUT/s20.jsonl'):
    d=json.loads(l); print('s20', d['value'], d['p50_latency_ms'], d['p99_latency_ms'])
d=json.load(open('$OUT/default.json')); print('s200', d['value'], d['p50_latency_ms'], d.get('vs_pytorch_eager_per_gpu'))"
