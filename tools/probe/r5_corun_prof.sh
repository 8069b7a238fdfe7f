# kernel times of the shipped throughput bench (4 batches in flight on the CU-partitioned halves)
export TMPDIR=/tmp
OUT=gpurun_out/r5corun
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace -d $OUT/prof -o run -- python3 bench.py --steps 200 --warmup 20 > $OUT/bench.json 2> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/bench.json
python3 tools/kernel_summary.py $OUT/prof --window 4500 --per 100 --top 40 > $OUT/summary.txt && cat $OUT/summary.txt
