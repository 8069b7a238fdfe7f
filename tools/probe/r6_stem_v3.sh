# Round 6: stem v3 (software-pipelined tile loop) -- bitwise test vs v2, kernel probe alone / 4
# co-running, then the bench A/B (MLS_STEM_VER=2 vs 3).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r6_stem_v3}
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -x -q -k stem --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -1 $OUT/pytest.log
for v in 2 3 2 3; do
  MLS_STEM_VER=$v timeout -k 10 120 python3 tools/probe/stem_pool_probe.py 2>/dev/null | sed "s/^{/{\"ver\": $v, /" >> $OUT/probe.jsonl || exit 1
done
cat $OUT/probe.jsonl
if [ -n "$BENCH" ]; then
  TAG=${TAG:-r6_stem_v3}_bench ROUNDS=${ROUNDS:-3} ARMS="v2:MLS_STEM_VER=2 v3:MLS_STEM_VER=3" bash tools/probe/r6_ab.sh
fi
