# 20-step window vs host staging threads (first-wave fill = 4 serial stagings), interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r5stage
mkdir -p $OUT
for r in 1 2 3; do
  for t in 4 8 12; do
    MLS_STAGE_THREADS=$t MLS_BENCH_TICKETS=$OUT/tickets_t${t}_$r.jsonl MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_t${t}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_t${t}_$r.json')); t=json.loads(open('$OUT/tickets_t${t}_$r.jsonl').readline())
print("threads", $t, "run", $r, d["value"], d["p50_latency_ms"], d["host_submit_ms_per_step"], "first tickets", t["tickets_ms"][:2])"
  done
done
