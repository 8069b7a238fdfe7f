mkdir -p gpurun_out/t8k
timeout -k 10 300 python3 -u -m pytest tests/test_transformer_ops_gpu.py -x -v --timeout 200 --timeout-method thread -k "8k" > gpurun_out/t8k/pytest.log 2>&1; rc=$?
tail -8 gpurun_out/t8k/pytest.log
exit $rc
