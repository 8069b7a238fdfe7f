# Full GPU suite + smoke + 1-GPU bench (the driver's round-end tiers), each bounded.
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest -x -q -m gpu --timeout 300 --timeout-method thread tests > $OUT/pytest_gpu.log 2>&1 \
  || { tail -40 $OUT/pytest_gpu.log; exit 1; }
tail -3 $OUT/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -2 $OUT/smoke.log
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > $OUT/bench1.json 2> $OUT/bench1.err || { tail -20 $OUT/bench1.err; exit 1; }
cat $OUT/bench1.json
