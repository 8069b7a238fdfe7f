# Kernel time split of one BERT-base B=128 S=128 fused forward (serial, 10 batches after warm-up).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${BP_OUT:-bert_prof}
mkdir -p $OUT
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py bert --batches 128 --inflight 1 --steps 10 --backends fused > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof --window 4000 --per 10 --top 25 > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
