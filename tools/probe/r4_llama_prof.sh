# Kernel split of Llama-3-8B prefill (B=8 x 512) + decode on the final tree: which kernels are not ours.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/llama_prof
mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py llama --batches 8 --prompt 512 --steps 10 > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof --top 40 > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
