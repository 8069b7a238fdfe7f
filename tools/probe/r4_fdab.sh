# fastdiv: skinny / Llama numerics, then throughput A/B against the base library on the same box.
export TMPDIR=/tmp
OUT=gpurun_out/fdab
mkdir -p $OUT
BASE=$PWD/tools/probe/alt_lib/libmls_base.so
timeout -k 10 500 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_skinny_packed_gpu.py tests/test_llama_tp_gpu.py tests/test_decode_pick_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
b() {  # name, env...
  name=$1; shift
  env "$@" timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/$name.json 2>> $OUT/bench.err || { tail -20 $OUT/bench.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/$name.json')); print('$name', d['value'], d['p50_latency_ms'])"
}
b base1 MLS_LIB_OVERRIDE=$BASE MLS_MEASURE_EAGER=0 && b new1 MLS_MEASURE_EAGER=0 && b base2 MLS_LIB_OVERRIDE=$BASE MLS_MEASURE_EAGER=0 && b new2 MLS_MEASURE_EAGER=0 && b base3 MLS_LIB_OVERRIDE=$BASE MLS_MEASURE_EAGER=0 && b new3 MLS_MEASURE_EAGER=0 || exit 1
l() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 1 8 --prompt 512 --steps 10 > $OUT/$name.jsonl 2>> $OUT/llama.err || { tail -20 $OUT/llama.err; return 1; }
  echo "$name"; cat $OUT/$name.jsonl
}
l lbase1 MLS_LIB_OVERRIDE=$BASE && l lnew1 && l lbase2 MLS_LIB_OVERRIDE=$BASE && l lnew2
