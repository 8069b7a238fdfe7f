# the in-forward-tuned concurrent table, and more batches in flight than masked streams, vs the default
export TMPDIR=/tmp
OUT=gpurun_out/r5infab
mkdir -p $OUT
for r in 1 2 3; do
  for v in base tab inf6 inf8; do
    unset MLS_TUNING_FILE; EXTRA=""
    [ $v = tab ] && export MLS_TUNING_FILE=tools/probe/tables/r5_corun_inforward.json
    [ $v = inf6 ] && EXTRA="--inflight 6"
    [ $v = inf8 ] && EXTRA="--inflight 8"
    MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 $EXTRA > $OUT/s20_${v}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "import json; d=json.load(open('$OUT/s20_${v}_$r.json')); print('$v', 's20 run', $r, d['value'], d['p50_latency_ms'])"
  done
done
for v in base tab inf6; do
  unset MLS_TUNING_FILE; EXTRA=""
  [ $v = tab ] && export MLS_TUNING_FILE=tools/probe/tables/r5_corun_inforward.json
  [ $v = inf6 ] && EXTRA="--inflight 6"
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 10 $EXTRA > $OUT/s200_${v}.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s200_${v}.json')); print('$v', 's200', d['value'], d['p50_latency_ms'])"
done
