# Whole-forward PMC totals of the fused ResNet-50 (bs=32), one rocprofv3 pass per counter group.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-fwd_pmc}
mkdir -p $OUT
i=0
for grp in "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum" \
           "GRBM_GUI_ACTIVE SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAVES"; do
  i=$((i+1))
  ITERS=3 timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/probe/forward_probe.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
  python3 tools/probe/forward_pmc_summary.py $OUT/p$i 3 > $OUT/p$i.summary.txt
done
cat $OUT/p*.summary.txt
