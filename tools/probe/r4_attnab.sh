# Flash attention with register double-buffered K/V tiles: numerics, then BERT engine and Llama prefill A/B.
export TMPDIR=/tmp
OUT=gpurun_out/${ATT_OUT:-attnab}
mkdir -p $OUT
BASE=$PWD/tools/probe/alt_lib/libmls_base.so
timeout -k 10 600 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_transformer_ops_gpu.py tests/test_e2e_gpu.py tests/test_models_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
b() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/$name.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; return 1; }
  echo "$name $(grep -o '"batch": [0-9]*\|"seq_per_s": [0-9.]*\|"throughput[a-z_]*": [0-9.]*' $OUT/$name.jsonl | tr '\n' ' ')"
}
l() {
  name=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/bench_models.py llama --batches 1 8 --prompt 512 --steps 10 > $OUT/$name.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; return 1; }
  echo "$name $(grep -o '"batch": [0-9]*\|"prefill_tok_s": [0-9.]*' $OUT/$name.jsonl | tr '\n' ' ')"
}
b bbase1 MLS_LIB_OVERRIDE=$BASE && b bnew1 && b bbase2 MLS_LIB_OVERRIDE=$BASE && b bnew2 && l lbase1 MLS_LIB_OVERRIDE=$BASE && l lnew1 && l lbase2 MLS_LIB_OVERRIDE=$BASE && l lnew2
