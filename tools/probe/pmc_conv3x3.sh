# MFMA / LDS / wait counters for the 3x3 convolutions (two rocprofv3 passes, counters only with
# --kernel-trace), summarised by tools/probe/pmc_summary.py
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc3
mkdir -p $OUT
LAYERS="${LAYERS:-layer1.1.conv2 layer2.1.conv2 layer3.1.conv2 layer4.1.conv2 layer1.0.conv3}"
i=0
for grp in "GRBM_GUI_ACTIVE SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES"; do
  i=$((i+1))
  ITERS=5 timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 $GRAFT_REPO_ROOT/tools/layer_probe.py $LAYERS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
echo done
