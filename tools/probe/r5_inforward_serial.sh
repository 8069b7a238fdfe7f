# in-forward tuning of the serial table (one batch, back-to-back forward replays), then serial A/B
export TMPDIR=/tmp
OUT=gpurun_out/r5infs
mkdir -p $OUT
L="layer1.0.conv1 layer2.0.conv2 layer2.0.dual layer2.1.conv1 layer3.0.conv2 layer3.0.dual layer3.1.conv1 layer3.1.conv3 layer3.2.conv1 layer3.2.conv3 layer3.3.conv1 layer3.3.conv3 layer3.4.conv1 layer3.4.conv3 layer3.5.conv1 layer3.5.conv3 layer4.0.conv1 layer4.0.conv2 layer4.0.dual layer4.1.conv1 layer4.1.conv3 layer4.2.conv1 layer4.2.conv3 fc"
timeout -k 10 900 python3 -u tools/inforward_tune.py --regime serial --reps 40 --layers $L --out $OUT/serial_table.json > $OUT/serial_tune.jsonl 2> $OUT/serial_tune.err || { tail -20 $OUT/serial_tune.err; exit 1; }
head -1 $OUT/serial_tune.jsonl; tail -1 $OUT/serial_tune.jsonl
for r in 1 2; do
  for t in shipped new; do
    if [ $t = new ]; then export MLS_TUNING_FILE=$OUT/serial_table.json; else unset MLS_TUNING_FILE; fi
    MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --serial --steps 100 --warmup 10 > $OUT/serial_${t}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/serial_${t}_$r.json')); print('$t', 'serial run', $r, d['value'], d['ms_per_step'], d['p50_latency_ms'])"
  done
done
