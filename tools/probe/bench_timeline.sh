# Fixed vs per-step cost of bench.py: elapsed at 20/40/80/160 steps (warmup 5) with per-batch
# submit/done times (MLS_BENCH_TICKETS), 2 rounds.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/timeline
mkdir -p $OUT
for r in 1 2; do
  for k in 20 40 80 160; do
    MLS_BENCH_TICKETS=$OUT/tickets.jsonl timeout -k 10 150 python3 bench.py --steps $k --warmup 5 >> $OUT/bench.jsonl 2>>$OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    tail -1 $OUT/bench.jsonl | cut -c1-200
  done
done
