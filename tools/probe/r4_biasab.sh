# Pipe-kernel bias staging after the prologue DMAs: numerics, serial forward A/B, 200-step bench A/B.
export TMPDIR=/tmp
OUT=gpurun_out/biasab
mkdir -p $OUT
BASE=$PWD/tools/probe/alt_lib/libmls_base.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_conv_pipe_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
OUT=gpurun_out/biasab bash tools/probe/r4_libab.sh || exit 1
b() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/$name.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['p50_latency_ms'])"
}
b bbase1 MLS_LIB_OVERRIDE=$BASE MLS_MEASURE_EAGER=0 && b bnew1 MLS_MEASURE_EAGER=0 && b bbase2 MLS_LIB_OVERRIDE=$BASE MLS_MEASURE_EAGER=0 && b bnew2 MLS_MEASURE_EAGER=0 && b bbase3 MLS_LIB_OVERRIDE=$BASE MLS_MEASURE_EAGER=0 && b bnew3 MLS_MEASURE_EAGER=0
