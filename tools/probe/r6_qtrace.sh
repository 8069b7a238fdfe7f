# Round 6: kernel traces with queue ids -- the bench with and without the early pull (prepull), and
# the engine gap probe's side-stream arm -- at the box's default hardware queues.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/r6_qtrace
mkdir -p $OUT
cd $R
timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/base -o run -- python3 bench.py --steps 40 --warmup 5 --measure-eager 0 > $OUT/base.json 2> $OUT/base.err || { tail -20 $OUT/base.err; exit 1; }
MLS_BENCH_PRESTAGE=1 MLS_PREPULL=1 timeout -k 10 240 rocprofv3 --kernel-trace --output-format csv -d $OUT/prepull -o run -- python3 bench.py --steps 40 --warmup 5 --measure-eager 0 > $OUT/prepull.json 2> $OUT/prepull.err || { tail -20 $OUT/prepull.err; exit 1; }
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/probe -o run -- python3 tools/probe/engine_gap_probe.py > $OUT/probe.txt 2> $OUT/probe.err || { tail -20 $OUT/probe.err; exit 1; }
for d in base prepull probe; do
  f=$(find $OUT/$d -name "*kernel_trace.csv" | head -1)
  python3 tools/probe/queue_trace.py "$f" --window 6 > $OUT/$d.queues.txt 2>&1 || exit 1
  rm -f "$f"
done
cat $OUT/base.json $OUT/prepull.json $OUT/probe.txt
head -12 $OUT/base.queues.txt; head -40 $OUT/prepull.queues.txt; head -40 $OUT/probe.queues.txt
