# stem v2 (fragment double buffer, stagger sweep) + head v2: numerics, stamps, timings
export TMPDIR=/tmp
OUT=gpurun_out/r5d2
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_ops_gpu.py -k "stem" tests/test_head_gpu.py > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for sg in 0 1300 2600; do
  MLS_STEM_STAGGER=$sg timeout -k 10 120 python3 tools/probe/stem_stamps.py 2>&1 | grep waves | sed "s/^/stagger $sg /"
  MLS_STEM_STAGGER=$sg timeout -k 10 120 python3 tools/probe/stem_pool_probe.py 2>&1 | grep concurrency | sed "s/^/stagger $sg /"
done
MLS_HEAD_V2=0 timeout -k 10 120 python3 tools/probe/head_probe.py 2>&1 | grep '"B"' | sed 's/^/head v1 /'
MLS_HEAD_V2=1 timeout -k 10 120 python3 tools/probe/head_probe.py 2>&1 | grep '"B"' | sed 's/^/head v2 /'
