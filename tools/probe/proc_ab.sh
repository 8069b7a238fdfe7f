# Process-level interleaved A/B of bench.py configurations on one box: each line of $CONFIGS is
# an env assignment prefix (e.g. "MLS_CHAIN=0"); ROUNDS rounds, the configs alternate inside each.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-proc_ab}
mkdir -p $OUT
ROUNDS=${ROUNDS:-3}
STEPS=${STEPS:-300}
for r in $(seq 1 $ROUNDS); do
  while IFS= read -r cfg; do
    [ -z "$cfg" ] && continue
    line=$(env $cfg timeout -k 10 150 python3 bench.py --steps $STEPS --warmup 30 $BENCH_ARGS 2>>$OUT/err.log) || { echo "FAILED: $cfg"; tail -20 $OUT/err.log; exit 1; }
    echo "{\"cfg\": \"$cfg\", \"round\": $r, \"bench\": $line}" >> $OUT/results.jsonl
    echo "$cfg r$r $(echo $line | python3 -c 'import json,sys; d=json.load(sys.stdin); print(d["value"], d["p50_latency_ms"])')"
  done <<< "$CONFIGS"
done
