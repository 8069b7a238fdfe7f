export TMPDIR=/tmp
OUT=gpurun_out/ar2
mkdir -p $OUT
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_custom_ar_gpu.py tests/test_llama_tp_gpu.py tests/test_decode_pick_gpu.py tests/test_continuous_device_gpu.py > $OUT/pytest.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest.log | tail -20; [ $rc -eq 0 ] || { grep -B5 -A60 "Error\b\|assert\|fused M=" $OUT/pytest.log | head -150; }; exit $rc
