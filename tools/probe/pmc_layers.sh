# Per-layer PMC counters for the conv kernel (one rocprofv3 pass per counter group).
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/pmc
mkdir -p $OUT
LAYERS="${LAYERS:-stem layer1.0.conv1 layer1.0.conv3 layer2.0.conv2 layer3.1.conv2 layer4.1.conv2}"
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY GRBM_GUI_ACTIVE SQ_INSTS_VALU" \
           "SQ_INSTS_MFMA SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_VALU_MFMA_BUSY_CYCLES" \
           "TCC_HIT_sum TCC_MISS_sum FETCH_SIZE" "WRITE_SIZE TCC_EA0_RDREQ_sum"; do
  i=$((i+1))
  ITERS=5 timeout -k 10 180 rocprofv3 --pmc $grp --kernel-trace --output-format csv -d $OUT/p$i -o run -- python3 tools/layer_probe.py $LAYERS > $OUT/p$i.log 2>&1 || { echo "pass $i failed"; tail -20 $OUT/p$i.log; exit 1; }
done
echo done
