export TMPDIR=/tmp
OUT=gpurun_out/prestage
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -60; exit $rc; }
for i in 1 2 3 4; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/t_on.jsonl timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/on.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  MLS_BENCH_PRESTAGE=0 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/off.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/on300.jsonl 2>> $OUT/err.log || exit 1
MLS_BENCH_PRESTAGE=0 MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/off300.jsonl 2>> $OUT/err.log || exit 1
python3 -c "
import json
for f in ['on','off','on300','off300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r], [x['host_submit_ms_per_step'] for x in r])
"
