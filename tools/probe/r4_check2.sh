export TMPDIR=/tmp
OUT=gpurun_out/check2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_continuous_device_gpu.py \
  tests/test_decode_pick_gpu.py tests/test_image_decode_gpu.py tests/test_llama_tp_gpu.py tests/test_e2e_gpu.py > $OUT/pytest.log 2>&1; rc=$?
grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -40
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\b\|assert" $OUT/pytest.log | head -120; exit $rc; }
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench_s20.json
MLS_MEASURE_EAGER=0 MLS_FUSED_HEAD=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_nohead.json 2>> $OUT/bench.err || exit 1
cat $OUT/bench_s20_nohead.json
bash tools/probe/pipe_pmc.sh
