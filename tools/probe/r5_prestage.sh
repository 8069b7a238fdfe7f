# prestaging the next batch while the slots are busy (MLS_BENCH_PRESTAGE=1), now that the bench polls its
# done events: 20-step A/B, interleaved
export TMPDIR=/tmp
OUT=gpurun_out/r5pre
mkdir -p $OUT
for r in 1 2 3 4 5; do
  for p in 0 1; do
    MLS_BENCH_PRESTAGE=$p MLS_BENCH_TICKETS=$OUT/tickets_p${p}_$r.jsonl MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_p${p}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_p${p}_$r.json'))
print('prestage', $p, 'run', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])"
  done
done
MLS_BENCH_PRESTAGE=1 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 200 > $OUT/s200_p1.json 2>> $OUT/err.log && MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 200 > $OUT/s200_p0.json 2>> $OUT/err.log && python3 -c "
import json
for p in (1,0):
    d=json.load(open('$OUT/s200_p%d.json'%p)); print('s200 prestage', p, d['value'], d['p50_latency_ms'])"
