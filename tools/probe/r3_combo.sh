# probe + selected GPU tests in one call (each step bounded, stop at the first failure)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-combo}
mkdir -p $OUT
if [ -n "$PROBE" ]; then
  timeout -k 10 500 python -u tools/gemm_tile_probe.py $PROBE > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -30 $OUT/probe.err; exit 1; }
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
  tail -5 $OUT/pytest.log
fi
