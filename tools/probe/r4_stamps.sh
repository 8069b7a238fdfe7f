# 20-step runs with per-submit host phases (slot wait / staging / enqueue) in the ticket log.
export TMPDIR=/tmp
OUT=gpurun_out/stamps
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3 4 5 6 7 8 9 10; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/s20_$r.json')); t=json.loads(open('$OUT/tickets_$r.jsonl').read().splitlines()[-1])
ph=[p for p in t['submit_phases_ms'] if p]; mx=[max(p[i] for p in ph) for i in range(3)]
print('s20', $r, d['value'], d['p99_latency_ms'], 'max slot-wait/stage/enqueue ms', mx)"
done
