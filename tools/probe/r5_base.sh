# Round-5 baseline: 5 driver-style 20-step runs (ticket + submit-phase logs), one 200-step run,
# and the serial forward's kernel summary.
export TMPDIR=/tmp
OUT=gpurun_out/r5base
mkdir -p $OUT
for r in 1 2 3 4 5; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/s20_$r.json')); t=json.loads(open('$OUT/tickets_$r.jsonl').read().splitlines()[-1])
ph=[p for p in t['submit_phases_ms'] if p]; mx=[max(p[i] for p in ph) for i in range(3)]
print('s20', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], 'max slot-wait/stage/enqueue ms', mx)"
done
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/s200.json 2>> $OUT/err.log && cat $OUT/s200.json
REGIME=serial GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial -- python3 tools/probe/forward_probe.py > $OUT/serial.log 2>&1 || { tail -20 $OUT/serial.log; exit 1; }
python3 tools/kernel_summary.py $OUT/serial --last-of stem_pool --per 30 --top 60 > $OUT/serial_summary.txt 2>&1
head -3 $OUT/serial_summary.txt
