# 4 masked slots with 4 vs 5 / 8 hardware queues per process (GPU_MAX_HW_QUEUES), interleaved.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/hwq
mkdir -p $OUT
for r in 1 2 3; do for q in 4 5 8; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/s20_q${q}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "q=$q s20 r=$r $(python3 -c "import json; d=json.load(open('$OUT/s20_q${q}_$r.json')); print(d['value'], d['p50_latency_ms'])")"
done; done
