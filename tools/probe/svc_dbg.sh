export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/svcdbg
mkdir -p $OUT
timeout -k 10 500 python3 -u -m pytest tests/test_engine_gpu.py tests/test_service_gpu.py -x -q -s --timeout 300 --timeout-method thread > $OUT/both.log 2>&1; echo "both rc $?"; grep -n -i "passed\|failed\|fault\|abort\|error" $OUT/both.log | head -20
