# is the 20-step window's first wave slowed by the idle gap of the pre-window gc.collect()? A/B
export TMPDIR=/tmp
OUT=gpurun_out/r5gc
mkdir -p $OUT
for r in 1 2 3 4 5; do
  for g in 0 1; do
    MLS_BENCH_GC_FIRST=$g MLS_BENCH_TICKETS=$OUT/tickets_g${g}_$r.jsonl MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_g${g}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_g${g}_$r.json')); t=json.loads(open('$OUT/tickets_g${g}_$r.jsonl').readline())
print('gc_first', $g, 'run', $r, d['value'], d['p50_latency_ms'], 'first submit', t['tickets_ms'][0], t['submit_phases_ms'][0], t['launch_us'][0])"
  done
done
