# bench client: completion-order reaping vs FIFO (MLS_BENCH_FIFO=1), interleaved.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/reap
mkdir -p $OUT
for r in 1 2 3; do for v in 0 1; do
  MLS_BENCH_FIFO=$v timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 > $OUT/s20_${v}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "fifo=$v s20 r=$r $(python3 -c "import json; d=json.load(open('$OUT/s20_${v}_$r.json')); print(d['value'], d['p50_latency_ms'], d['p99_latency_ms'])")"
done; done
for r in 1 2; do for v in 0 1; do
  MLS_BENCH_FIFO=$v timeout -k 10 300 python3 bench.py --steps 200 --warmup 20 > $OUT/s200_${v}_$r.json 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  echo "fifo=$v s200 r=$r $(python3 -c "import json; d=json.load(open('$OUT/s200_${v}_$r.json')); print(d['value'], d['p50_latency_ms'], d['p99_latency_ms'])")"
done; done
