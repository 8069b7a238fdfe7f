# Round 6 measurement campaign on the final tree: smoke, default bench (200 steps + same-run eager),
# 5 driver-form runs, BERT engine, HTTP through the native front end, in-situ kernel summary.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_campaign}
mkdir -p $OUT
cd $R
timeout -k 10 300 python3 -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { tail -20 $OUT/smoke.log; exit 1; }
tail -1 $OUT/smoke.log
timeout -k 10 400 python3 bench.py > $OUT/default.json 2> $OUT/default.err || { tail -20 $OUT/default.err; exit 1; }
cut -c1-400 $OUT/default.json
: > $OUT/s20.jsonl
for r in 1 2 3 4 5; do
  MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 >> $OUT/s20.jsonl 2>> $OUT/s20.err || { tail -20 $OUT/s20.err; exit 1; }
done
python3 -c "
import json
for l in open('$OUT/s20.jsonl'):
    d=json.loads(l); print('s20', d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])"
if [ -z "$SKIP_SECONDARY" ]; then
for i in 1 2; do
  timeout -k 10 400 python3 -u tools/bench_models.py bert --batches 32 64 128 --backends fused >> $OUT/bert.jsonl 2>> $OUT/bert.err || { tail -20 $OUT/bert.err; exit 1; }
done
cut -c1-250 $OUT/bert.jsonl
hb() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python3 -u tools/http_bench.py "$@" --frontend native --duration 6 --warmup 2 --ready-timeout 200 > $OUT/http_$name.jsonl 2> $OUT/http_$name.err || { tail -20 $OUT/http_$name.err; return 1; }
  echo "$name $(python3 -c "
import json
for l in open('$OUT/http_$name.jsonl'):
    d=json.loads(l); print(d['conns'], d['requests_per_s'], d['p50_ms'], end=' | ')")"
}
hb resnet_raw --model resnet50 --conns 128 256 || exit 1
hb resnet_jpeg --model resnet50 --jpeg --conns 128 256 || exit 1
hb bert_text --model bert --text --conns 128 256 || exit 1
fi
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prof -o run -- python3 bench.py --steps 120 --warmup 10 --measure-eager 0 > $OUT/prof.json 2> $OUT/prof.err || { tail -20 $OUT/prof.err; exit 1; }
f=$(find $OUT/prof -name "*kernel_trace.csv" | head -1)
python3 tools/kernel_summary.py "$f" --last-of stem_pool --per 100 --top 30 > $OUT/kernel_summary.txt || exit 1
rm -f "$f"
head -12 $OUT/kernel_summary.txt
