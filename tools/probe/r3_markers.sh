# roctx marker traces: ResNet-50 serving bench (bench.py, 5 in flight) and Llama
# decode, MLS_TRACE=1, rocprofv3 --marker-trace --kernel-trace (no counters), summarised.
export TMPDIR=/tmp MLS_TRACE=1
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-markers}
mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $OUT/resnet -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 20 --warmup 5 > $OUT/resnet.log 2>&1 || { tail -20 $OUT/resnet.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/probe/marker_summary.py $OUT/resnet > $OUT/resnet_markers.txt && head -20 $OUT/resnet_markers.txt
cd /tmp && timeout -k 10 400 rocprofv3 --marker-trace --kernel-trace --output-format csv -d $OUT/llama -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py llama --batches 8 --steps 10 > $OUT/llama.log 2>&1 || { tail -20 $OUT/llama.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/probe/marker_summary.py $OUT/llama > $OUT/llama_markers.txt && head -20 $OUT/llama_markers.txt
