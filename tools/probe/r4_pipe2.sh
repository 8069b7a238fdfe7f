export TMPDIR=/tmp
OUT=gpurun_out/pipe2
mkdir -p $OUT
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pipe_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
timeout -k 10 400 python -u tools/probe/pipe_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
grep '"best": true' $OUT/probe.jsonl
for i in 1 2 3; do
  MLS_MEASURE_EAGER=0 MLS_BENCH_TICKETS=$OUT/tickets.jsonl timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$i.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench_s20_$i.json
done
MLS_DIST_BACKEND=gloo MLS_MEASURE_EAGER=0 timeout -k 10 600 python3 bench.py --gpus 8 --steps 20 --warmup 5 > $OUT/bench_gloo8.json 2> $OUT/bench_gloo8.err || { tail -30 $OUT/bench_gloo8.err; exit 1; }
cat $OUT/bench_gloo8.json
