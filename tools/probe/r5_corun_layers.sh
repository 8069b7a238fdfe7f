# per-layer co-running kernel times (4 batches on 2 CU-masked halves) for one table: $1 = shipped |
# flush (tools/probe/tables/r5_conc_flush_merged.json).  rocprofv3 segfaults in __cxa_finalize AFTER
# writing its database when the process used CU-masked streams, so one table per call.
export TMPDIR=/tmp
OUT=gpurun_out/r5corunl
mkdir -p $OUT
t=$1
if [ "$t" = flush ]; then export MLS_TUNING_FILE=tools/probe/tables/r5_conc_flush_merged.json; fi
ITERS=20 timeout -k 10 300 rocprofv3 --kernel-trace -d $OUT/prof_$t -o run -- python3 tools/probe/corun_layers.py > $OUT/run_$t.log 2>&1
python3 tools/probe/corun_layers.py --report $OUT/prof_$t/run_results.db > $OUT/layers_$t.txt && tail -1 $OUT/layers_$t.txt
