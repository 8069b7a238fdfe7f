# End-of-round profiles: serial kernel summary of the shipped forward + whole-forward PMC totals.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/finalprof
mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --serial --steps 20 --warmup 5 > $OUT/prof_serial.log 2>&1 || { tail -20 $OUT/prof_serial.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof_serial --window 940 --per 20 --top 40 > $OUT/prof_serial_summary.txt 2>&1; head -8 $OUT/prof_serial_summary.txt
sed -i "s#OUT=\$GRAFT_REPO_ROOT/gpurun_out/fwd_pmc#OUT=\$GRAFT_REPO_ROOT/gpurun_out/finalprof/fwd_pmc#" tools/probe/forward_pmc.sh
bash tools/probe/forward_pmc.sh
