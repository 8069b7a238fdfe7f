# end-of-round check on the final tree: full GPU suite + smoke, default bench, 3 driver-style runs
export TMPDIR=/tmp
OUT=gpurun_out/r5final2
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread -x > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 300 python3 bench.py > $OUT/default.json 2> $OUT/default.err || { tail -20 $OUT/default.err; exit 1; }
cat $OUT/default.json
for r in 1 2 3; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/s20_$r.json')); print('s20 run', $r, d['value'], d['p50_latency_ms'], d['host_submit_ms_per_step'])"
done
