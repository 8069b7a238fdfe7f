# Pipe-kernel magic-number divisions: numerics, serial forward per-kernel profile, s20 bench x3.
export TMPDIR=/tmp
OUT=gpurun_out/magic${TAG}
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pipe_gpu.py ${EXTRA_TESTS} > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
REGIME=serial GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial -- python3 tools/probe/forward_probe.py > $OUT/serial.log 2>&1 || { tail -20 $OUT/serial.log; exit 1; }
python3 tools/kernel_summary.py $OUT/serial --last-of stem_pool --per 30 --top 45 > $OUT/serial_summary.txt 2>&1
head -1 $OUT/serial_summary.txt
for i in 1 2 3; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$i.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  python3 -c "import json; d=json.load(open('$OUT/bench_s20_$i.json')); print('s20', d['value'], d['p50_latency_ms'])"
done
