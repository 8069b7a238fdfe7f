# HTTP (native front end) ResNet-50: partitioned engine with 5 / 6 slots over 4 masked streams vs
# unpartitioned 5 slots; bench default; then the in-situ kernel trace of the partitioned bench.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/httppart2
mkdir -p $OUT
hb() {  # name, env...
  local name=$1; shift
  env "$@" timeout -k 10 300 python3 -u tools/http_bench.py --model resnet50 --frontend native --conns 128 256 --duration 6 --warmup 2 --ready-timeout 200 > $OUT/$name.jsonl 2> $OUT/$name.err || { tail -20 $OUT/$name.err; exit 1; }
  echo "$name $(python3 -c "
import json
for l in open('$OUT/$name.jsonl'):
    d=json.loads(l); print(d['conns'], d['requests_per_s'], d['p50_ms'], end=' | ')")"
}
hb p2_if5 CU_PARTITION=2 INFLIGHT=5
hb p0_if5 CU_PARTITION=0 INFLIGHT=5
hb p2_if6 CU_PARTITION=2 INFLIGHT=6
hb p2_if8 CU_PARTITION=2 INFLIGHT=8
timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/bench_s200.json 2>$OUT/b.err || { tail $OUT/b.err; exit 1; }
python3 -c "import json; d=json.load(open('$OUT/bench_s200.json')); print('bench s200', d['value'], d['p50_latency_ms'], d['config']['inflight'])"
bash tools/probe/prof_partitioned.sh
