# Quick flagship check: bench at the driver's settings x2, steady state, serial kernel summary.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/quick
mkdir -p $OUT
for i in 1 2; do
  timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/bench_s20_$i.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench_s20_$i.json
done
timeout -k 10 300 python3 bench.py --gpus 1 --steps 300 --warmup 20 > $OUT/bench_s300.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
cat $OUT/bench_s300.json
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_serial -o run -- python3 $GRAFT_REPO_ROOT/bench.py --serial --steps 20 --warmup 5 > $OUT/prof_serial.log 2>&1 || { tail -20 $OUT/prof_serial.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof_serial --window 940 --per 20 --top 60 > $OUT/prof_serial_summary.txt 2>&1; head -30 $OUT/prof_serial_summary.txt
