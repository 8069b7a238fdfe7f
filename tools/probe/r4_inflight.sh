export TMPDIR=/tmp
OUT=gpurun_out/inflight
mkdir -p $OUT
for rep in 1 2; do
for inf in 4 5 6 8; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$inf.jsonl timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --inflight $inf >> $OUT/if$inf.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
done
python3 -c "
import json
for inf in (4,5,6,8):
    r=[json.loads(l) for l in open('$OUT/if%d.jsonl'%inf)]
    print(inf, [x['value'] for x in r], [x['p50_latency_ms'] for x in r], [x['p99_latency_ms'] for x in r])
"
