# serial ResNet-50 forward kernel summary (graph replays, serial table)
export TMPDIR=/tmp
OUT=gpurun_out/r5prof${TAG}
mkdir -p $OUT
REGIME=serial GRAPH=1 ITERS=40 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/serial -- python3 tools/probe/forward_probe.py > $OUT/serial.log 2>&1 || { tail -20 $OUT/serial.log; exit 1; }
python3 tools/kernel_summary.py $OUT/serial --last-of stem_pool --per 30 --top 60 > $OUT/serial_summary.txt 2>&1
head -3 $OUT/serial_summary.txt; grep -E "stem|head|fc_" $OUT/serial_summary.txt
