# Round 6: hardware counters of the native tile GEMM (cfg 15) vs hipBLASLt on two Llama-3-8B
# prefill shapes (4096 rows: O 4096x4096x4096, down 4096x4096x14336).  One counter pass per rocprofv3
# run (block limits: <= 8 SQ, <= 4 TCC), kernel trace filtered to the two GEMMs.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${TAG:-r6_gemm_pmc}
mkdir -p $OUT
cd $R
timeout -s KILL 60 rocprofv3 --list-avail > $OUT/avail.txt 2>&1 || true
grep -oE "(SQ|TCC|TA|TCP)_[A-Z0-9_]+" $OUT/avail.txt | sort -u > $OUT/avail_names.txt || true
P="python3 $R/tools/gemm_tile_probe.py --shapes llama_o llama_down --cfgs 15 --conc 1 --iters 5"
run_pass() {  # $1 = name, rest = counters
  local n=$1; shift
  timeout -s KILL 150 rocprofv3 --pmc "$@" --kernel-include-regex "gemm_tile|Cijk" --output-format csv -d $OUT/$n -o run -- $P > $OUT/$n.log 2>&1 || { echo "pass $n failed"; tail -5 $OUT/$n.log; return 1; }
}
run_pass a SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE || exit 1
run_pass b SQ_INSTS_LDS SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_SALU || exit 1
run_pass c TCC_HIT_sum TCC_MISS_sum || exit 1
python3 $R/tools/probe/pmc_kernel_means.py $OUT/a $OUT/b $OUT/c > $OUT/summary.txt && cat $OUT/summary.txt
