# masked streams destroyed at exit (ops.partition.release_masked_streams): a plain 20-step bench must
# still exit 0, and a rocprofv3 kernel trace of the partitioned bench must no longer segfault at exit
export TMPDIR=/tmp
OUT=gpurun_out/r5exit
mkdir -p $OUT
MLS_MEASURE_EAGER=0 timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $OUT/plain.json 2> $OUT/plain.err; echo "plain rc=$?"; cat $OUT/plain.json
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 bench.py --steps 200 --warmup 20 > $OUT/prof.json 2> $OUT/prof.err; echo "rocprof rc=$?"; cat $OUT/prof.json
ls -la $OUT/prof
