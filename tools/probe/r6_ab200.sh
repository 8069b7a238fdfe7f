# Round 6: interleaved A/B at 200 steps (ROUNDS pairs) plus 20-step driver-form pairs.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r6_ab200}
mkdir -p $OUT
: > $OUT/bench.jsonl
run_arm() {  # $1 = arm spec, $2 = steps, $3 = warmup
  local name=${1%%:*} envs=${1#*:}
  local e=""
  [ "$envs" != "$1" ] && e=$(echo "$envs" | tr ',' ' ')
  env $e timeout -k 10 300 python3 bench.py --gpus 1 --steps $2 --warmup $3 --measure-eager 0 > $OUT/b.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; return 1; }
  python3 -c "import json; d=json.load(open('$OUT/b.json')); d['arm']='$name'; print(json.dumps(d))" >> $OUT/bench.jsonl
}
for i in $(seq 1 ${ROUNDS:-3}); do
  for arm in $ARMS; do run_arm "$arm" 200 20 || exit 1; done
  for arm in $ARMS; do run_arm "$arm" 20 5 || exit 1; done
done
python3 -c "
import json
for l in open('$OUT/bench.jsonl'):
    d=json.loads(l); print(d['arm'], d['steps'], d['value'], d['p50_latency_ms'], d['p99_latency_ms'], d['host_submit_ms_per_step'])
"
