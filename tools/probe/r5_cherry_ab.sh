# A/B of the concurrent table with 5 co-run-verified flushed picks (tools/probe/tables/r5_conc_cherry.json)
# vs the shipped one: 20-step window (x4 interleaved) and 200 steps
export TMPDIR=/tmp
OUT=gpurun_out/r5cherryab
mkdir -p $OUT
C=tools/probe/tables/r5_conc_cherry.json
for r in 1 2 3 4; do
  for t in shipped flush; do
    if [ $t = flush ]; then export MLS_TUNING_FILE=$C; else unset MLS_TUNING_FILE; fi
    MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${t}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/s20_${t}_$r.json')); print('$t', 's20 run', $r, d['value'], d['p50_latency_ms'])"
  done
done
for r in 1 2; do
  for t in shipped flush; do
    if [ $t = flush ]; then export MLS_TUNING_FILE=$C; else unset MLS_TUNING_FILE; fi
    MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 > $OUT/s200_${t}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/s200_${t}_$r.json')); print('$t', 's200 run', $r, d['value'], d['p50_latency_ms'])"
  done
done
