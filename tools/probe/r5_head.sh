# head finisher rewrite: tests + serial profile
export TMPDIR=/tmp
OUT=gpurun_out/r5head
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_head_gpu.py tests/test_ops_gpu.py -k "head or topk or softmax" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
TAG=head bash tools/probe/r5_serial_prof.sh
