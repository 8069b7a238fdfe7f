# fastdiv in the conv kernels: numerics of every conv path, then the same-box library A/B.
export TMPDIR=/tmp
OUT=gpurun_out/fastdiv
mkdir -p $OUT
timeout -k 10 700 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py tests/test_chain_gpu.py tests/test_conv_pipe_gpu.py tests/test_models_gpu.py tests/test_e2e_gpu.py tests/test_head_gpu.py > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A30 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
OUT=gpurun_out/fastdiv bash tools/probe/r4_libab.sh && REGIME=concurrent OUT=gpurun_out/fastdiv_c bash tools/probe/r4_libab.sh
