# SDMA-free engine I/O (MLS_PULL_H2D=8: H2D pull + D2H push kernels in the slot graph) vs the SDMA
# copies: engine numerics, then interleaved 20-step driver-style runs with ticket logs, 200 steps.
export TMPDIR=/tmp
OUT=gpurun_out/r5stallab
mkdir -p $OUT
MLS_PULL_H2D=8 timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_engine_gpu.py > $OUT/pytest_engine_pull.log 2>&1 || { tail -30 $OUT/pytest_engine_pull.log; exit 1; }
tail -1 $OUT/pytest_engine_pull.log
N=${RUNS:-12}
for r in $(seq 1 $N); do
  for arm in sdma pull8 spin pull8spin; do
    case $arm in pull8) E="MLS_PULL_H2D=8";; spin) E="MLS_EVENT_SPIN_US=20000";; pull8spin) E="MLS_PULL_H2D=8 MLS_EVENT_SPIN_US=20000";; *) E="MLS_PULL_H2D=0";; esac
    env $E MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets_${arm}_$r.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${arm}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_${arm}_$r.json')); t=json.loads(open('$OUT/tickets_${arm}_$r.jsonl').read().splitlines()[-1])
ph=t['submit_phases_ms']; lu=t['launch_us']
worst=max(range(len(ph)), key=lambda i: sum(ph[i]) if ph[i] else 0)
print('$arm', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'], 'worst', worst, ph[worst], lu[worst])"
  done
done
for arm in sdma pull8 spin pull8spin; do
  case $arm in pull8) E="MLS_PULL_H2D=8";; spin) E="MLS_EVENT_SPIN_US=20000";; pull8spin) E="MLS_PULL_H2D=8 MLS_EVENT_SPIN_US=20000";; *) E="MLS_PULL_H2D=0";; esac
  env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/s200_$arm.json 2>> $OUT/err.log && python3 -c "import json; d=json.load(open('$OUT/s200_$arm.json')); print('s200 $arm', d['value'], d['p50_latency_ms'], d['p99_latency_ms'])"
done
