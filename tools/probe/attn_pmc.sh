# PMC counters of the decode-attention kernel at batch 128 (two passes: SQ instruction mix / waits,
# then HBM fetch bytes), kernel-filtered.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/attn_pmc
mkdir -p $OUT
cd /tmp
timeout -s KILL 240 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_SALU --kernel-include-regex decode_attn --output-format csv -d $OUT/p1 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py llama --batches 128 --steps 3 > $OUT/p1.log 2>&1 || { tail -5 $OUT/p1.log; exit 1; }
timeout -s KILL 240 rocprofv3 --pmc FETCH_SIZE TCC_HIT_sum --kernel-include-regex decode_attn --output-format csv -d $OUT/p2 -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py llama --batches 128 --steps 3 > $OUT/p2.log 2>&1 || { tail -5 $OUT/p2.log; exit 1; }
ls $OUT/p1 $OUT/p2
