# BERT-base fused forward, engine-like (5 batches in flight), kernel-time split: native tile GEMMs vs
# the hipBLASLt A/B arm.  B=${B:-32}.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-bert_prof_ab}
mkdir -p $OUT
for impl in native blas; do
  cd /tmp && MLS_GEMM_IMPL=$impl timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/$impl -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py bert --batches ${B:-32} --inflight 5 --steps 20 --backends fused > $OUT/$impl.log 2>&1 || { tail -20 $OUT/$impl.log; exit 1; }
  cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/$impl --window 4000 --per 20 --top 14 > $OUT/summary_$impl.txt 2>&1
  grep seq_per_s $OUT/$impl.log | tail -1; head -16 $OUT/summary_$impl.txt | cut -c1-150
done
