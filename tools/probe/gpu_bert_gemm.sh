# BERT projection GEMMs: hipBLASLt vs native, then hipBLASLt under PyTorch TunableOp.
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python tools/probe/bert_gemm_probe.py > gpurun_out/bert_gemm.jsonl 2> gpurun_out/bert_gemm.err && \
PROBE_TAG=tunableop PYTORCH_TUNABLEOP_ENABLED=1 PYTORCH_TUNABLEOP_TUNING=1 PYTORCH_TUNABLEOP_FILENAME=gpurun_out/tunableop_bert.csv \
  timeout -k 10 400 python tools/probe/bert_gemm_probe.py >> gpurun_out/bert_gemm.jsonl 2>> gpurun_out/bert_gemm.err && \
timeout -k 10 300 python tools/bench_models.py bert --batches 32 --inflight 5 --steps 200 --backends fused >> gpurun_out/bert_gemm.jsonl 2>> gpurun_out/bert_gemm.err
