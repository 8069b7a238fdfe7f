# Kernel trace of the default (partitioned) bench: per-kernel in-situ durations.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/profpart2
mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 100 --warmup 10 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof --window 4700 --per 100 --top 40 > $OUT/summary.txt 2>&1; head -45 $OUT/summary.txt
