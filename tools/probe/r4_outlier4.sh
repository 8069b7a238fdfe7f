# 20-step outlier hunt on the final tree: 8 runs with per-batch submit / done timelines and phase stamps.
export TMPDIR=/tmp
OUT=gpurun_out/outlier4
mkdir -p $OUT
for r in 1 2 3 4 5 6 7 8; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s20_$r.json')); print('s20', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])"
done
