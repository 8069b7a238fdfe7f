# Batch-32 decode: kernel breakdown (packed on), and the bench at batch 24 / 32 with packed on / off.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/b32
mkdir -p $OUT
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- python3 tools/bench_models.py llama --batches 32 --steps 10 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
python3 tools/probe/decode_step_breakdown.py $OUT/kt/run_kernel_trace.csv | tee $OUT/breakdown_b32.txt
for cfg in "MLS_PACKED_DECODE=1" "MLS_PACKED_DECODE=0"; do
  env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --batches 24 32 --steps 30 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  sed "s/^{/{\"cfg\": \"$cfg\", /" $OUT/b.tmp | grep -v init_s | tee -a $OUT/bench.jsonl
done
