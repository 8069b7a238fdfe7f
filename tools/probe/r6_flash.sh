# Round 6: Llama-shaped causal GQA prefill attention (D = 128) alone -- time per call and counters.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_flash}
mkdir -p $OUT
cd $R
timeout -k 10 120 python3 tools/probe/flash_probe.py --batches 1 8 --tag "${ARM:-base}" | tee -a $OUT/time.jsonl || exit 1
[ "${PMC:-1}" = 1 ] || exit 0
P="python3 $R/tools/probe/flash_probe.py --batches 8 --iters 3"
run_pass() {
  local n=$1; shift
  timeout -s KILL 100 rocprofv3 --pmc "$@" --kernel-include-regex "flash_fwd" --output-format csv -d $OUT/$n -o run -- $P > $OUT/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $OUT/$n.log; return 1; }
}
run_pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run_pass b SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_INSTS_VALU_TRANS_F32 || run_pass b SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU SQ_WAIT_INST_LDS || exit 1
run_pass c TCC_HIT_sum TCC_MISS_sum || exit 1
python3 $R/tools/probe/pmc_kernel_means.py $OUT/a $OUT/b $OUT/c > $OUT/summary.txt && cat $OUT/summary.txt
