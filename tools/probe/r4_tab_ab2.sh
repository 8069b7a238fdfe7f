export TMPDIR=/tmp
OUT=gpurun_out/tabab2
mkdir -p $OUT
for i in 1 2 3; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/conc.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=tools/probe/alt_tables/resnet50_r4_partitioned_retune.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/ser.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/conc300.jsonl 2>> $OUT/err.log || exit 1
MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=tools/probe/alt_tables/resnet50_r4_partitioned_retune.json timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/ser300.jsonl 2>> $OUT/err.log || exit 1
python3 -c "
import json
for f in ['conc','ser','conc300','ser300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r])
"
