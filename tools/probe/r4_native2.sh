export TMPDIR=/tmp
OUT=gpurun_out/native2
mkdir -p $OUT
for i in 1 2; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/on300.jsonl 2>> $OUT/err.log || exit 1
  MLS_NATIVE_LAUNCH=0 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/off300.jsonl 2>> $OUT/err.log || exit 1
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/on.jsonl 2>> $OUT/err.log || exit 1
  MLS_NATIVE_LAUNCH=0 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/off.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for f in ['on','off','on300','off300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r], [x['host_submit_ms_per_step'] for x in r])
"
