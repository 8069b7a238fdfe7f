# Full GPU check of the tree: pytest -m gpu, smoke(), and the flagship bench at the driver's settings.
OUT=$GRAFT_REPO_ROOT/gpurun_out/round_check
mkdir -p $OUT
timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$i.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench_s20_$i.json
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 300 --warmup 20 > $OUT/bench_s300.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench_s300.json
