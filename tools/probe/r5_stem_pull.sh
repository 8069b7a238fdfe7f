# stem v2 numerics + timing (v1 vs v2), then zero-copy H2D A/B on the 20-step bench.
export TMPDIR=/tmp
OUT=gpurun_out/r5sp
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "stem" > $OUT/pytest_stem.log 2>&1 || { tail -30 $OUT/pytest_stem.log; exit 1; }
tail -1 $OUT/pytest_stem.log
MLS_STEM_V2=0 timeout -k 10 120 python3 tools/probe/stem_pool_probe.py 2>&1 | grep concurrency | sed 's/^/v1 /'
MLS_STEM_V2=1 timeout -k 10 120 python3 tools/probe/stem_pool_probe.py 2>&1 | grep concurrency | sed 's/^/v2 /'
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > $OUT/pytest_engine.log 2>&1 || { tail -30 $OUT/pytest_engine.log; exit 1; }
tail -1 $OUT/pytest_engine.log
MLS_PULL_H2D=16 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > $OUT/pytest_engine_pull.log 2>&1 || { tail -30 $OUT/pytest_engine_pull.log; exit 1; }
tail -1 $OUT/pytest_engine_pull.log
for r in 1 2 3 4 5 6 7 8; do
  for arm in sdma pull16; do
    if [ $arm = pull16 ]; then E="MLS_PULL_H2D=16"; else E="MLS_PULL_H2D=0"; fi
    env $E MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_${arm}_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${arm}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_${arm}_$r.json')); t=json.loads(open('$OUT/tickets_${arm}_$r.jsonl').read().splitlines()[-1])
ph=t['submit_phases_ms']; lu=t['launch_us']
worst=max(range(len(ph)), key=lambda i: sum(ph[i]) if ph[i] else 0)
print('$arm', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], 'worst', worst, ph[worst], lu[worst])"
  done
done
for arm in sdma pull16; do
  if [ $arm = pull16 ]; then E="MLS_PULL_H2D=16"; else E="MLS_PULL_H2D=0"; fi
  env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/s200_$arm.json 2>> $OUT/err.log && python3 -c "import json; d=json.load(open('$OUT/s200_$arm.json')); print('s200 $arm', d['value'], d['p50_latency_ms'], d['p99_latency_ms'])"
done
