export TMPDIR=/tmp
OUT=gpurun_out/chain
mkdir -p $OUT
for rep in 1 2; do
for arm in default nochain chainl3; do
  case $arm in default) E="";; nochain) E="MLS_CHAIN=0";; chainl3) E="MLS_CHAIN_L3=1";; esac
  env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/$arm.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
done
for arm in default nochain chainl3; do
  case $arm in default) E="";; nochain) E="MLS_CHAIN=0";; chainl3) E="MLS_CHAIN_L3=1";; esac
  env $E MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/${arm}300.jsonl 2>> $OUT/err.log || exit 1
done
python3 -c "
import json
for f in ['default','nochain','chainl3','default300','nochain300','chainl3300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r])
"
