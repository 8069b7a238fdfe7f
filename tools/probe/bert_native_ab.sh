# BERT-base engine (B=32, S=128, 5 in flight): native tuned-tile projections vs hipBLASLt, interleaved
# process-level A/B, plus the BERT GPU numerics tests.
OUT=$GRAFT_REPO_ROOT/gpurun_out/bertab
mkdir -p $OUT
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_models_gpu.py -k bert > $OUT/test.log 2>&1 || { tail -30 $OUT/test.log; exit 1; }
tail -2 $OUT/test.log
for r in 1 2 3; do
  for cfg in "MLS_BERT_NATIVE_GEMM=1" "MLS_BERT_NATIVE_GEMM=0"; do
    env $cfg timeout -k 10 300 python3 tools/bench_models.py bert --backends fused --batches 32 --seqs 128 --steps 200 > $OUT/b.tmp 2> $OUT/b.err || { tail -20 $OUT/b.err; exit 1; }
    sed "s/^{/{\"cfg\": \"$cfg\", \"round\": $r, /" $OUT/b.tmp | tee -a $OUT/bench.jsonl
  done
done
