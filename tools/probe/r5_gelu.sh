# tanh-form GELU in the GEMM epilogues: GELU numerics tests, the FFN-up GEMM timing, BERT engine
export TMPDIR=/tmp
OUT=gpurun_out/r5gelu
mkdir -p $OUT
timeout -k 10 400 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/ -m gpu -k "gelu or linear_dispatch or bert or gemm_tile or ln_fold or skinny or gemm" > $OUT/tests.log 2>&1 || { tail -30 $OUT/tests.log; exit 1; }
tail -2 $OUT/tests.log
PYTHONPATH=. timeout -k 10 240 python3 -u tools/probe/ln_fold_probe.py 16384 > $OUT/probe.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
cat $OUT/probe.jsonl
for r in 1 2; do
  timeout -k 10 300 python3 -u tools/bench_models.py bert --batches 32 128 --backends fused > $OUT/bench_$r.jsonl 2>> $OUT/err.log || { tail -20 $OUT/err.log; exit 1; }
  cat $OUT/bench_$r.jsonl
done
