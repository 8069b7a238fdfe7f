# Full GPU suite (driver-style) + smoke on the current tree
export TMPDIR=/tmp
OUT=gpurun_out/r5full
mkdir -p $OUT
timeout -k 10 1000 python3 -u -m pytest tests/ -q -m gpu --timeout 300 --timeout-method thread -x > $OUT/pytest.log 2>&1; rc=$?
tail -15 $OUT/pytest.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
