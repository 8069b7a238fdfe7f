# probe + selected GPU tests in one call (each step bounded, stop at the first failure)
export TMPDIR=/tmp
OUT=gpurun_out/${TAG:-combo}
mkdir -p $OUT
if [ -n "$PROBE" ]; then
  timeout -k 10 500 python -u tools/gemm_tile_probe.py $PROBE > $OUT/probe.jsonl 2> $OUT/probe.err || { tail -30 $OUT/probe.err; exit 1; }
fi
if [ -n "$TESTS" ]; then
  timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread $TESTS > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
  tail -5 $OUT/pytest.log
fi
if [ -n "$BERT" ]; then  # fused BERT-base throughput: native tile GEMMs vs hipBLASLt A/B
  for impl in native blas; do
    MLS_GEMM_IMPL=$impl timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --seqs 128 --steps 40 --inflight 5 --backends fused > $OUT/bert_$impl.jsonl 2>> $OUT/bert.err || { tail -20 $OUT/bert.err; exit 1; }
    cat $OUT/bert_$impl.jsonl
  done
fi
if [ -n "$BENCH" ]; then
  timeout -k 10 400 python3 -u bench.py --steps 20 --warmup 5 > $OUT/bench.json 2> $OUT/bench.err || { tail -20 $OUT/bench.err; exit 1; }
  cat $OUT/bench.json
fi
