# Item-2 check on the final tree: 10 consecutive driver-style 20-step runs on one box, then the
# default 200-step bench and the 8-rank gloo rehearsal (8 ranks sharing this box's one GPU)
export TMPDIR=/tmp
OUT=gpurun_out/${R5F_OUT:-r5final}
mkdir -p $OUT
for r in 1 2 3 4 5 6 7 8 9 10; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/s20_$r.json'))
print('s20', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], d['config']['partition_mode'])"
done
timeout -k 10 600 python3 bench.py > $OUT/default.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/default.json
MLS_DIST_BACKEND=gloo MLS_MEASURE_EAGER=0 timeout -k 10 600 python3 bench.py --gpus 8 --steps 20 --warmup 5 > $OUT/gloo8.json 2> $OUT/gloo8.err || { tail -20 $OUT/gloo8.err; exit 1; }
cat $OUT/gloo8.json
