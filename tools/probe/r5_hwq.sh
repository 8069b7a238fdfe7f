# hardware queues per process (GPU_MAX_HW_QUEUES, HIP default 4) x batches in flight, 20-step window
export TMPDIR=/tmp
OUT=gpurun_out/r5hwq
mkdir -p $OUT
for r in 1 2; do
  for cfg in "4 4" "8 4" "8 6" "8 8"; do
    set -- $cfg
    GPU_MAX_HW_QUEUES=$1 INFLIGHT=$2 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_q$1_i$2_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_q$1_i$2_$r.json'))
print('hwq', $1, 'inflight', $2, 'run', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], d['config']['inflight'])"
  done
done
