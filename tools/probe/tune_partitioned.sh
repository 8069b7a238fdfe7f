# Re-tune the ResNet-50 B=32 conv table with 4 copies co-running on 2 CU partitions (the engine's
# default regime), then A/B the bench: shipped table vs the new one.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/tune
mkdir -p $OUT
MLS_TUNE_PARTITIONS=2 timeout -k 10 1000 python3 -u -m mlmicroservicetemplate_amd.ops.autotune --batch 32 --concurrency 4 --no-torch --out $OUT/resnet50_b32_p2c4.json > $OUT/tune.log 2>&1 || { tail -20 $OUT/tune.log; exit 1; }
tail -1 $OUT/tune.log
for r in 1 2; do
  for t in shipped new; do
    if [ $t = new ]; then export MLS_TUNING_FILE=$OUT/resnet50_b32_p2c4.json; else unset MLS_TUNING_FILE; fi
    timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/b_${t}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    echo "$t $r $(python3 -c "import json; d=json.load(open('$OUT/b_${t}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
  done
done
