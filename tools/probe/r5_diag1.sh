# stem v2 stamps + numerics, head probe, pull kernel widths, pull4/pull8 vs SDMA 20-step A/B
export TMPDIR=/tmp
OUT=gpurun_out/r5d1
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "stem" > $OUT/pytest_stem.log 2>&1 || { tail -30 $OUT/pytest_stem.log; exit 1; }
tail -1 $OUT/pytest_stem.log
timeout -k 10 120 python3 tools/probe/stem_stamps.py 2>&1 | grep waves
timeout -k 10 120 python3 tools/probe/head_probe.py 2>&1 | grep '"B"'
timeout -k 10 120 python3 tools/probe/h2d_pull_probe.py 2>&1 | grep bytes
for r in 1 2 3 4 5 6; do
  for arm in sdma pull4 pull8; do
    case $arm in pull4) E="MLS_PULL_H2D=4";; pull8) E="MLS_PULL_H2D=8";; *) E="MLS_PULL_H2D=0";; esac
    env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_${arm}_$r.json 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    python3 -c "
import json; d=json.load(open('$OUT/s20_${arm}_$r.json'))
print('$arm', $r, d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])"
  done
done
