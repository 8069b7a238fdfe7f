export TMPDIR=/tmp
OUT=gpurun_out/l4ab
mkdir -p $OUT
for i in 1 2 3; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/new.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  MLS_MEASURE_EAGER=0 MLS_TUNING_FILE=tools/probe/alt_tables/resnet50_r4_before_l4pipe.json timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 >> $OUT/old.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
done
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --steps 300 --warmup 20 >> $OUT/new300.jsonl 2>> $OUT/err.log || exit 1
python3 -c "
import json
for f in ['new','old','new300']:
    r=[json.loads(l) for l in open('$OUT/'+f+'.jsonl')]
    print(f, [x['value'] for x in r], [x['p50_latency_ms'] for x in r])
"
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -- python3 bench.py --steps 60 --warmup 5 --measure-eager 0 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/kernel_summary.py $OUT/prof --window 3000 --per 60 --top 40 > $OUT/prof_summary.txt 2>&1; head -45 $OUT/prof_summary.txt
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_custom_ar_gpu.py tests/test_llama_tp_gpu.py > $OUT/pytest_ar.log 2>&1; rc=$?; grep -E "PASSED|FAILED|ERROR|passed|failed" $OUT/pytest_ar.log | tail -20; exit $rc
