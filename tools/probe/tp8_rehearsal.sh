mkdir -p gpurun_out/tp8
timeout -k 10 600 python3 -u -m pytest tests/test_llama_tp_gpu.py tests/test_custom_ar_gpu.py -x -v --timeout 400 --timeout-method thread > gpurun_out/tp8/pytest.log 2>&1; rc=$?
tail -30 gpurun_out/tp8/pytest.log
exit $rc
