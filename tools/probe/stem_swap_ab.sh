# Stem epilogue A/B: numerics tests, kernel probe and bench with MLS_STEM_SWAP=0/1.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/stem
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest tests/test_ops_gpu.py -k "stem" -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
for sw in 0 1; do MLS_STEM_SWAP=$sw timeout -k 10 120 python3 tools/probe/stem_pool_probe.py > $OUT/probe_$sw.jsonl 2>&1 || { tail $OUT/probe_$sw.jsonl; exit 1; }; echo "swap=$sw"; cat $OUT/probe_$sw.jsonl; done
for r in 1 2; do for sw in 0 1; do
  MLS_STEM_SWAP=$sw timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/b_${sw}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "swap=$sw r=$r $(python3 -c "import json; d=json.load(open('$OUT/b_${sw}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
done; done
