# Round-3 GPU check: new GPU tests (RCCL world-1, exact bench config e2e, engine roctx ranges),
# the 1-GPU bench, a 4-rank bench through bench.py's own launcher (gloo, shared GPU), then the
# full GPU suite.  Each step bounded; stop at the first failure.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-r3a}
mkdir -p $OUT
set -o pipefail
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_rccl_gpu.py \
  tests/test_engine_gpu.py tests/test_ops_gpu.py::test_resnet50_fused_matches_reference > $OUT/pytest_new.log 2>&1 \
  || { tail -40 $OUT/pytest_new.log; exit 1; }
tail -3 $OUT/pytest_new.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { tail -20 $OUT/bench1.err; exit 1; }
cat $OUT/bench1.json
MLS_DIST_BACKEND=gloo timeout -k 10 400 python bench.py --gpus 4 --steps 20 --warmup 5 > $OUT/bench4_gloo.json 2> $OUT/bench4.err || { tail -20 $OUT/bench4.err; exit 1; }
cat $OUT/bench4_gloo.json
if [ "${FULL:-1}" = 1 ]; then
  timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest_gpu.log 2>&1 \
    || { tail -40 $OUT/pytest_gpu.log; exit 1; }
  tail -3 $OUT/pytest_gpu.log
fi
