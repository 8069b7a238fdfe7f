export TMPDIR=/tmp
OUT=gpurun_out/outlier3
mkdir -p $OUT
for i in 1 2 3 4 5 6 7 8 9 10 11 12; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/on.jsonl 2>> $OUT/err.log || exit 1
  MLS_NATIVE_LAUNCH=0 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/off.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for f in ['on','off']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    v=[x['value'] for x in r]
    print(f, v, 'median', sorted(v)[len(v)//2], [x['host_submit_ms_per_step'] for x in r])
"
