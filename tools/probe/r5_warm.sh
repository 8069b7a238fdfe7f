# does the 20-step window run below steady state because the GPU is still ramping? warmup sweep
export TMPDIR=/tmp
OUT=gpurun_out/r5warm
mkdir -p $OUT
for r in 1 2; do
  for w in 5 50 200; do
    MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup $w > $OUT/s20_w${w}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_w${w}_$r.json'))
print('warmup', $w, 'run', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'])"
  done
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 100 --warmup 5 > $OUT/s100_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/s100_$r.json'))
print('steps 100 warmup 5 run', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'])"
done
