# engine tests, CDLL vs PyDLL enqueue A/B (20 steps)
export TMPDIR=/tmp
OUT=gpurun_out/r5c3
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py tests/test_service_gpu.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for r in 1 2 3 4; do
  for arm in cdll pydll; do
    if [ $arm = pydll ]; then E="MLS_ENQUEUE_HOLD_GIL=1"; else E="MLS_ENQUEUE_HOLD_GIL=0"; fi
    env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${arm}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_${arm}_$r.json'))
print('$arm', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])"
  done
done
