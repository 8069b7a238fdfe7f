# H2D pull workgroups (MLS_PULL_H2D) in the 20-step window, interleaved
export TMPDIR=/tmp
OUT=gpurun_out/r5pullwg
mkdir -p $OUT
for r in 1 2 3; do
  for w in 8 4 16; do
    MLS_PULL_H2D=$w MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_w${w}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/s20_w${w}_$r.json')); print('wg', $w, 'run', $r, d['value'], d['p50_latency_ms'])"
  done
done
for w in 8 16; do
  MLS_PULL_H2D=$w MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 > $OUT/s200_w${w}.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s200_w${w}.json')); print('s200 wg', $w, d['value'], d['p50_latency_ms'])"
done
