export TMPDIR=/tmp
OUT=gpurun_out/stage
mkdir -p $OUT
nproc > $OUT/nproc.txt; python3 -c "import os; print(len(os.sched_getaffinity(0)))" >> $OUT/nproc.txt
for rep in 1 2; do
for t in 1 4 8 12; do
  MLS_STAGE_THREADS=$t MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$t.jsonl timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/t$t.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
done
cat $OUT/nproc.txt
python3 -c "
import json
for t in (1,4,8,12):
    r=[json.loads(l) for l in open('$OUT/t%d.jsonl'%t)]
    tk=[json.loads(l) for l in open('$OUT/tickets_%d.jsonl'%t)]
    print(t, [x['value'] for x in r], [x['p50_latency_ms'] for x in r], [x['host_submit_ms_per_step'] for x in r], [k['tickets_ms'][0][0] for k in tk], [k['tickets_ms'][3][0] for k in tk])
"
