# Interleaved A/B of the SDMA-copy stall: default vs HSA_ENABLE_SDMA_GANG=0 vs a copy-engine
# pre-warm in the engine warm-up (MLS_COPY_PREWARM=64), 20-step driver-style runs.
export TMPDIR=/tmp
OUT=gpurun_out/r5sdma2
mkdir -p $OUT
N=${RUNS:-20}
for r in $(seq 1 $N); do
  for arm in default nogang prewarm; do
    case $arm in
      nogang) E="HSA_ENABLE_SDMA_GANG=0";;
      prewarm) E="MLS_COPY_PREWARM=64";;
      *) E="MLS_NOOP=1";;
    esac
    env $E MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_${arm}_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${arm}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_${arm}_$r.json')); t=json.loads(open('$OUT/tickets_${arm}_$r.jsonl').read().splitlines()[-1])
ph=t['submit_phases_ms']; lu=t['launch_us']
worst=max(range(len(ph)), key=lambda i: sum(ph[i]) if ph[i] else 0)
print('$arm', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], 'worst', worst, ph[worst], lu[worst])"
  done
done
