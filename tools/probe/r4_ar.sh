export TMPDIR=/tmp
OUT=gpurun_out/ar
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_custom_ar_gpu.py tests/test_llama_tp_gpu.py > $OUT/pytest_ar.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_ar.log | tail -20; [ $rc -eq 0 ] || { grep -B5 -A40 "Error\b\|assert" $OUT/pytest_ar.log | head -100; }; exit $rc
