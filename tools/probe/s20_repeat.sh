# Repeatability of the driver-style run (20 steps): 5 back-to-back bench processes + one 200-step.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/rep
mkdir -p $OUT
for r in 1 2 3 4 5; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/s20_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "s20 $r $(python3 -c "import json; d=json.load(open('$OUT/s20_$r.json')); print(d['value'], d['p50_latency_ms'], d['p99_latency_ms'])")"
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 200 --warmup 20 > $OUT/s200.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
echo "s200 $(python3 -c "import json; d=json.load(open('$OUT/s200.json')); print(d['value'], d['p50_latency_ms'])")"
