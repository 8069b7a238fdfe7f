# 20-step window: second stream of each CU partition on a thinned mask (MLS_SLOT_THIN=k drops every
# (the MLS_SLOT_THIN option was measured slower and removed from engine/worker.py; kept as the record)
# k-th CU) so the two batches of a half desynchronize -- interleaved A/B
export TMPDIR=/tmp
OUT=gpurun_out/r5thin
mkdir -p $OUT
for r in 1 2 3; do
  for k in 0 8 4; do
    MLS_SLOT_THIN=$k MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_k${k}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/s20_k${k}_$r.json')); print('thin', $k, 'run', $r, d['value'], d['p50_latency_ms'])"
  done
done
for k in 0 8; do
  MLS_SLOT_THIN=$k MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 5 > $OUT/s200_k${k}.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s200_k${k}.json')); print('s200 thin', $k, d['value'], d['p50_latency_ms'])"
done
