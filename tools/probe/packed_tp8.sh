# Packed decode GEMMs on one emulated TP=8 rank (collectives stubbed) vs the row-major path.
OUT=$GRAFT_REPO_ROOT/gpurun_out/packed_tp8
mkdir -p $OUT
for cfg in "MLS_PACKED_DECODE=0" "MLS_PACKED_DECODE=1" ${EXTRA_CFGS}; do
  env $cfg timeout -k 10 300 python3 tools/bench_models.py llama --emulate-tp 8 --batches 1 8 --steps 30 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
  sed "s/^{/{\"cfg\": \"$cfg\", /" $OUT/b.tmp | tee -a $OUT/bench.jsonl
done
