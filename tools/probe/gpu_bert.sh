# BERT-base B=32 S=128 at 3 / 5 / 8 batches in flight (fused vs eager), then a kernel trace of fused
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
for n in 3 5 8; do
  timeout -k 10 300 python -u tools/bench_models.py bert --batches 32 --inflight $n --steps 60 >> gpurun_out/bert_inflight.jsonl 2>> gpurun_out/bert_inflight.err || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_bert -o run -- python3 tools/bench_models.py bert --batches 32 --inflight 1 --steps 10 --backends fused > gpurun_out/prof_bert.log 2>&1
