# LayerNorm folding (round 5): GPU numerics, BERT throughput folded vs unfolded, serial kernel split.
export TMPDIR=/tmp
OUT=$GRAFT_REPO_ROOT/gpurun_out/r5lnfold
mkdir -p $OUT
cd $GRAFT_REPO_ROOT
PYTHONPATH=. timeout -k 10 240 python3 -u tools/probe/ln_fold_probe.py > $OUT/probe.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/probe.jsonl
timeout -k 10 400 python3 -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_ln_fold_gpu.py \
  "tests/test_models_gpu.py::test_bert_fused_matches_reference" "tests/test_e2e_gpu.py::test_bert_b128_s128_engine_vs_fp32" \
  > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -3 $OUT/tests.log
for r in 1 2; do
  for f in 1 0; do
    MLS_BERT_LN_FOLD=$f timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused \
      > $OUT/bench_f${f}_$r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
    echo "fold=$f run $r"; cat $OUT/bench_f${f}_$r.jsonl
  done
done
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_models.py bert --batches 128 --inflight 1 --steps 10 --backends fused > $OUT/prof.log 2>&1 || { tail -20 $OUT/prof.log; exit 1; }
cd $GRAFT_REPO_ROOT && python3 tools/kernel_summary.py $OUT/prof --window 4000 --per 10 --top 25 > $OUT/summary.txt 2>&1; cat $OUT/summary.txt
