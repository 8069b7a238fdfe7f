# PMC passes over tools/probe/pipe_pmc_run.py (counters only with --kernel-trace; one block's
# limits per pass), summarised by tools/probe/pmc_summary.py; plus the box's counter list.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pipe_pmc
mkdir -p $OUT
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do
  i=$((i+1))
  cd /tmp && timeout -s KILL 120 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/probe/pipe_pmc_run.py > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -5 $OUT/p$i.log; }
done
cd /tmp && timeout -s KILL 60 rocprofv3 -L > $OUT/counters_list.txt 2>&1 || true
cd $GRAFT_REPO_ROOT && python3 tools/probe/pmc_summary.py $OUT > $OUT/summary.txt; cat $OUT/summary.txt
