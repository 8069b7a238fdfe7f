# Re-tune both ResNet tables on the fastdiv kernels, then A/B each against the shipped table.
export TMPDIR=/tmp
OUT=gpurun_out/tune3
mkdir -p $OUT
MLS_TUNE_PARTITIONS=2 timeout -k 10 600 python3 -u -m mlmicroservicetemplate_amd.ops.autotune --batch 32 --concurrency 4 --no-torch --out $OUT/part.json > $OUT/tune_part.jsonl 2> $OUT/tune_part.err || { tail -5 $OUT/tune_part.err; exit 1; }
timeout -k 10 600 python3 -u -m mlmicroservicetemplate_amd.ops.autotune --batch 32 --concurrency 1 --no-torch --out $OUT/ser.json > $OUT/tune_ser.jsonl 2> $OUT/tune_ser.err || { tail -5 $OUT/tune_ser.err; exit 1; }
python3 - <<'PY'
import json
for ship_f, new_f, out_f in [('resnet50_gfx950_b32.json', 'part.json', 'merged_part.json'), ('resnet50_gfx950_b32_serial.json', 'ser.json', 'merged_ser.json')]:
    ship = json.load(open('mlmicroservicetemplate_amd/ops/tuned/' + ship_f))
    new = json.load(open('gpurun_out/tune3/' + new_f))
    out, n = {}, 0
    for k, v in ship.items():
        if k in new and isinstance(v, dict) and (new[k]["best_cfg"], new[k]["best_splitk"]) != (v.get("best_cfg"), v.get("best_splitk")):
            n += 1
        out[k] = new.get(k, v)
    json.dump(out, open('gpurun_out/tune3/' + out_f, 'w'), indent=1)
    print(out_f, "changed", n)
PY
for i in 1 2 3; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/ship.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=$OUT/merged_part.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/new.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
for i in 1 2; do
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 >> $OUT/ship200.jsonl 2>> $OUT/err.log || exit 1
MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=$OUT/merged_part.json timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 >> $OUT/new200.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for f in ['ship','new','ship200','new200']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r])
"
run() {  # name, env...
  name=$1; shift
  env "$@" REGIME=serial GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$name -- python3 tools/probe/forward_probe.py > $OUT/$name.log 2>&1 || { tail -20 $OUT/$name.log; return 1; }
  python3 tools/kernel_summary.py $OUT/$name --last-of stem_pool --per 30 --top 45 > $OUT/${name}_summary.txt 2>&1
  echo "$name $(head -1 $OUT/${name}_summary.txt)"
}
run ser_ship && run ser_new MLS_TUNING_FILE=$OUT/merged_ser.json && run ser_ship2 && run ser_new2 MLS_TUNING_FILE=$OUT/merged_ser.json
