export TMPDIR=/tmp
OUT=gpurun_out/chainbm
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_chain_gpu.py > $OUT/pytest.log 2>&1; rc=$?; tail -2 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -A30 "Error\b" $OUT/pytest.log | head -40; exit $rc; }
for rep in 1 2; do
for arm in default bm64 cw32; do
  case $arm in default) E="";; bm64) E="MLS_CHAIN_L2_BM=64";; cw32) E="MLS_CHAIN_L2_CW=32";; esac
  env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/$arm.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
done
for arm in default bm64; do
  case $arm in default) E="";; bm64) E="MLS_CHAIN_L2_BM=64";; esac
  env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/${arm}300.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for f in ['default','bm64','cw32','default300','bm64300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r])
"
