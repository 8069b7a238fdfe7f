export TMPDIR=/tmp
OUT=gpurun_out/c4prof
mkdir -p $OUT
CONC=4 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -- python3 tools/probe/forward_probe.py > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
python3 tools/kernel_summary.py $OUT/prof --last-of stem_pool --per 120 --top 45 > $OUT/summary.txt 2>&1
head -48 $OUT/summary.txt
