export TMPDIR=/tmp
OUT=gpurun_out/tune2
mkdir -p $OUT
MLS_TUNE_PARTITIONS=2 timeout -k 10 1000 python3 -u -m mlmicroservicetemplate_amd.ops.autotune --batch 32 --concurrency 4 --no-torch --iters 50 --out $OUT/part50.json > $OUT/tune.jsonl 2> $OUT/tune.err || { tail -5 $OUT/tune.err; exit 1; }
tail -1 $OUT/tune.jsonl
python3 - <<'PY'
import json
ship=json.load(open('mlmicroservicetemplate_amd/ops/tuned/resnet50_gfx950_b32.json'))
new=json.load(open('gpurun_out/tune2/part50.json'))
out={}
n=0
for k,v in ship.items():
    if k in new and (new[k]["best_cfg"],new[k]["best_splitk"])!=(v["best_cfg"],v["best_splitk"]): n+=1
    out[k]=new.get(k,v)
json.dump(out, open('gpurun_out/tune2/merged.json','w'), indent=1)
print("changed", n)
PY
for i in 1 2 3; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/ship.jsonl 2>> $OUT/err.log || exit 1
  MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=$OUT/merged.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/new.jsonl 2>> $OUT/err.log || exit 1
done
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/ship300.jsonl 2>> $OUT/err.log || exit 1
MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=$OUT/merged.json timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/new300.jsonl 2>> $OUT/err.log || exit 1
python3 -c "
import json
for f in ['ship','new','ship300','new300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r])
"
