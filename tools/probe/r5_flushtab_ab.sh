# A/B of the L2-flushed re-tune (tools/probe/tables/r5_*_flush_merged.json) vs the shipped tables:
# 20-step window (x3 interleaved), 200 steps, and the serial forward
export TMPDIR=/tmp
OUT=gpurun_out/r5flushab
mkdir -p $OUT
C=tools/probe/tables/r5_conc_flush_merged.json
S=tools/probe/tables/r5_serial_flush_merged.json
for r in 1 2 3; do
  for t in shipped flush; do
    if [ $t = flush ]; then export MLS_TUNING_FILE=$C; else unset MLS_TUNING_FILE; fi
    MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${t}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/s20_${t}_$r.json')); print('$t', 's20 run', $r, d['value'], d['p50_latency_ms'])"
  done
done
for t in shipped flush; do
  if [ $t = flush ]; then export MLS_TUNING_FILE=$C; else unset MLS_TUNING_FILE; fi
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 > $OUT/s200_${t}.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s200_${t}.json')); print('$t', 's200', d['value'], d['p50_latency_ms'])"
done
for t in shipped flush; do
  if [ $t = flush ]; then export MLS_TUNING_FILE=$S; else unset MLS_TUNING_FILE; fi
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --serial --steps 100 --warmup 10 > $OUT/serial_${t}.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/serial_${t}.json')); print('$t', 'serial', d['value'], d['ms_per_step'], d['p50_latency_ms'])"
done
