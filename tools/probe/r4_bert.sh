export TMPDIR=/tmp
OUT=gpurun_out/bert
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_e2e_gpu.py tests/test_transformer_ops_gpu.py tests/test_models_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -60; exit $rc; }
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/bert.jsonl 2> $OUT/bert.err || { tail -20 $OUT/bert.err; exit 1; }
cat $OUT/bert.jsonl
timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused >> $OUT/bert.jsonl 2>> $OUT/bert.err && tail -2 $OUT/bert.jsonl
