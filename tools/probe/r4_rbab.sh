# Row-block RMSNorm (decode) with batched loads: numerics, then Llama decode / serving A/B.
export TMPDIR=/tmp
OUT=gpurun_out/${RB_OUT:-rbab}
mkdir -p $OUT
BASE=$PWD/tools/probe/alt_lib/libmls_base.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_models_gpu.py tests/test_continuous_device_gpu.py tests/test_kv_pages_gpu.py tests/test_llama_tp_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
l() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 32 128 --prompt 128 --steps 20 > $OUT/$name.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; return 1; }
  echo "$name $(grep -o '"batch": [0-9]*\|"decode_ms_per_step": [0-9.]*' $OUT/$name.jsonl | tr '\n' ' ')"
}
S="tools/bench_models.py llama-serve --batches 256 --kv-pages 769 --requests 1024 --prompt 128 --new 64"
s() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 -u $S > $OUT/$name.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; return 1; }
  echo "$name $(grep -o '"tokens_per_s": [0-9.]*' $OUT/$name.jsonl)"
}
l lbase1 MLS_LIB_OVERRIDE=$BASE && l lnew1 && l lbase2 MLS_LIB_OVERRIDE=$BASE && l lnew2 && s sbase1 MLS_LIB_OVERRIDE=$BASE && s snew1 && s sbase2 MLS_LIB_OVERRIDE=$BASE && s snew2
