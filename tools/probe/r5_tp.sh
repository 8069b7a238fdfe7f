# custom all-reduce (incl. the fused-stall case) and the TP serving tests (TP=8 tokens vs TP=1)
export TMPDIR=/tmp
OUT=gpurun_out/r5tp
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_custom_ar_gpu.py > $OUT/ar.log 2>&1; rc=$?
grep -E "passed|failed|fused stall|Error" $OUT/ar.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest -x -v -s --timeout 600 --timeout-method thread tests/test_llama_tp_gpu.py -k "serving" > $OUT/tp.log 2>&1; rc=$?
grep -E "passed|failed|rank .*iterations|Error|assert" $OUT/tp.log | tail -20
exit $rc
