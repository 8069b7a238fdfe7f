export TMPDIR=/tmp
OUT=gpurun_out/full5
mkdir -p $OUT
timeout -k 10 1500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?
tail -5 $OUT/pytest.log
[ $rc -eq 0 ] || { grep -B5 -A40 "Error\b\|assert" $OUT/pytest.log | head -80; exit $rc; }
timeout -k 10 400 python3 bench.py > $OUT/bench_default.json 2> $OUT/bench_default.err || { tail -20 $OUT/bench_default.err; exit 1; }
cat $OUT/bench_default.json
timeout -k 10 300 python3 -c "import __graft_entry__ as e; e.smoke(); print('smoke ok')" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
