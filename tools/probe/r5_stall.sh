# 20-step driver-style runs with per-HIP-call enqueue times in the ticket log: which call a
# multi-ms submit stall sits in.
export TMPDIR=/tmp
OUT=gpurun_out/r5stall${TAG}
mkdir -p $OUT
N=${RUNS:-12}
for r in $(seq 1 $N); do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $BENCH_ARGS > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/s20_$r.json')); t=json.loads(open('$OUT/tickets_$r.jsonl').read().splitlines()[-1])
ph=t['submit_phases_ms']; lu=t['launch_us']
worst=max(range(len(ph)), key=lambda i: sum(ph[i]) if ph[i] else 0)
print('s20', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], 'worst submit', worst, ph[worst], 'launch_us', lu[worst], 'first', t['tickets_ms'][0])"
done
