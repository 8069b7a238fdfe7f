# BERT with the tuned GEMM routing: numerics at the bench shape, then bench A/B (tables on / off).
set -o pipefail
mkdir -p gpurun_out
rm -f gpurun_out/bert_tuned.jsonl
timeout -k 10 300 python -u -m pytest tests/test_models_gpu.py -x -q --timeout 120 --timeout-method thread -k bert > gpurun_out/bert_tuned_test.log 2>&1 && \
timeout -k 10 300 python tools/bench_models.py bert --batches 32 --inflight 5 --steps 300 >> gpurun_out/bert_tuned.jsonl 2>> gpurun_out/bert_tuned.err && \
MLS_BLAS_TUNING=0 timeout -k 10 300 python tools/bench_models.py bert --batches 32 --inflight 5 --steps 300 --backends fused | sed 's/^{/{"blas_tuning": 0, /' >> gpurun_out/bert_tuned.jsonl 2>> gpurun_out/bert_tuned.err && \
timeout -k 10 300 python tools/bench_models.py bert --batches 32 --inflight 1 --steps 300 --backends fused >> gpurun_out/bert_tuned.jsonl 2>> gpurun_out/bert_tuned.err
