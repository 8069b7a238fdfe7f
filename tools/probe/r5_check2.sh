# engine/head/stem GPU tests, serial profile, default bench x5 (20 steps) + 200 steps
export TMPDIR=/tmp
OUT=gpurun_out/r5c2
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_head_gpu.py tests/test_ops_gpu.py tests/test_service_gpu.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
TAG=c2 bash tools/probe/r5_serial_prof.sh || exit 1
for r in 1 2 3 4 5; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  python3 -c "
import json; d=json.load(open('$OUT/s20_$r.json'))
print('s20', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])"
done
timeout -k 10 300 python3 bench.py --gpus 1 > $OUT/s200.json 2>> $OUT/err.log && cat $OUT/s200.json
