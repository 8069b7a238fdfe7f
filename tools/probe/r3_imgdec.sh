# GPU image decode: tests, timing probe, per-kernel split
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-imgdec}
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_image_decode_gpu.py > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python -u tools/image_decode_probe.py > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
cat $OUT/probe.jsonl
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/image_decode_probe.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/probe/marker_summary.py $OUT/prof | tail -9
